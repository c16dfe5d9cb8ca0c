"""The C ring (include/mm_ring.h, host/mm_ring.c): frame-sharded streaming with
one RCCL ncclSend/ncclRecv per step, driven by the C host (mm_cli --ring-*).

CPU: the library loads, links RCCL and exports every symbol mm_ring.h declares.
GPU: at world 1 the ring shifts the state to and from the same rank through
RCCL every step; the output must be bitwise the single-process stream.  The
multi-rank step logic (rank 0's carry of the state received one step earlier,
both state slots reused, the next step's shift posted ahead) runs at world 2,
3 and 8 through the ring's test-only local transport (host/mm_ring_local.h:
rank threads of one process on one GPU, device copies instead of RCCL, which
refuses two ranks on one device) — `mm_cli --ring-local G`.  RCCL itself at
world > 1 runs only on an 8-GPU node.
"""
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "phase-based-motion-manipulation_amd")
LIB = os.path.join(PKG, "lib", "libmm_ring.so")
CLI = os.path.join(PKG, "bin", "mm_cli")
HDR = os.path.join(ROOT, "include", "mm_ring.h")


def header_symbols():
    txt = re.sub(r"/\*.*?\*/", "", open(HDR).read(), flags=re.S)
    return sorted(set(re.findall(r"\b(mm_ring_[a-z_]+)\s*\(", txt)))


def test_ring_library_exports_header_symbols():
    syms = header_symbols()
    assert syms == ["mm_ring_core_library", "mm_ring_create", "mm_ring_destroy", "mm_ring_get_id",
                    "mm_ring_halo_frames", "mm_ring_last_error", "mm_ring_step", "mm_ring_step_halo"]
    out = subprocess.run(["nm", "-D", "--defined-only", LIB], capture_output=True, text=True,
                         check=True).stdout
    exported = {ln.split()[-1] for ln in out.splitlines() if " T " in ln}
    assert set(syms) <= exported
    deps = subprocess.run(["ldd", LIB], capture_output=True, text=True, check=True).stdout
    assert "librccl" in deps and "libmm355" in deps


def test_ring_rejects_bad_arguments_without_gpu():
    import ctypes
    L = ctypes.CDLL(LIB)
    L.mm_ring_create.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_int,
                                 ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                 ctypes.c_int, ctypes.POINTER(ctypes.c_void_p)]
    out = ctypes.c_void_p()
    idb = (ctypes.c_ubyte * 128)()
    assert L.mm_ring_create(1, 0, idb, 0, None, 64, 48, 4, 0, ctypes.byref(out)) == -1
    assert L.mm_ring_create(0, 0, idb, 0, None, 64, 48, 4, 0, ctypes.byref(out)) == -1
    L.mm_ring_step.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                               ctypes.c_void_p, ctypes.c_void_p]
    assert L.mm_ring_step(None, 0, None, None, None, None) == -1


def _checksums(txt):
    return [(int(a), int(b)) for a, b in re.findall(r"^frame (\d+) (\d+)$", txt, flags=re.M)]


@pytest.mark.gpu
def test_c_ring_world1_equals_single_stream(tmp_path):
    """mm_cli --ring-world 1: 4 steps of 12 frames at 256x144 through the RCCL
    self-ring == mm_cli over the same 48 frames in one process (bitwise)."""
    common = ["-w", "256", "-h", "144", "-n", "48", "-b", "12", "-l", "5", "-s", "25", "--checksum"]
    env = dict(os.environ, NCCL_DEBUG="WARN")
    one = subprocess.run([CLI] + common, capture_output=True, text=True, timeout=120, env=env)
    assert one.returncode == 0, one.stderr
    ring = subprocess.run([CLI] + common + ["--ring-world", "1", "--ring-rank", "0",
                                            "--ring-id", str(tmp_path / "ring.id")],
                          capture_output=True, text=True, timeout=180, env=env)
    assert ring.returncode == 0, ring.stdout + ring.stderr
    a, b = _checksums(one.stdout), _checksums(ring.stdout)
    assert len(a) == 48 and a == b


def _bench(args):
    import json
    import sys
    env = dict(os.environ, NCCL_DEBUG="WARN", PYTHONUNBUFFERED="1")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, env=env, cwd=ROOT,
                       capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    return json.loads([x for x in r.stdout.splitlines() if x.startswith("{")][-1])


@pytest.mark.gpu
def test_bench_c_ring_world1_1080p_equals_single_rank():
    """bench.py's N>1 ring path is the C ring: at world 1
    (--ring-self) every step's state goes through libmm_ring's RCCL
    send/receive to the same rank; at 1920x1080 the per-frame output
    checksums of 3 steps x 8 frames equal the plain single-rank stream."""
    common = ["--checksum", "--frames-per-step", "8", "--steps", "2", "--warmup", "1"]
    one = _bench(common)
    ring = _bench(common + ["--ring-self"])
    assert one["frames"] == ring["frames"] == [0, 23]
    assert not one["inputs_wrapped"] and not ring["inputs_wrapped"]
    assert one["checksums"] == ring["checksums"]
    line = _bench(["--ring-self", "--frames-per-step", "16", "--steps", "2", "--warmup", "1",
                   "--no-cpu-baseline", "--drop-in-frames", "0"])
    assert "C host RCCL ring" in line["config"]["parallelism"], line["config"]
    assert line["value"] > 0


def _cli(args, timeout):
    env = dict(os.environ, NCCL_DEBUG="WARN")
    r = subprocess.run([CLI] + args, capture_output=True, text=True, timeout=timeout, env=env)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    return r.stdout


def test_ring_local_rejects_uneven_stream():
    """--ring-local needs the stream to be whole steps of G chunks (checked
    before any device work)."""
    r = subprocess.run([CLI, "-w", "64", "-h", "48", "-n", "10", "-b", "4", "--ring-local", "2"],
                       capture_output=True, text=True, timeout=60)
    assert r.returncode == 2 and "multiple of G * batch" in r.stderr


def test_ring_local_symbols_exported():
    out = subprocess.run(["nm", "-D", "--defined-only", LIB], capture_output=True, text=True,
                         check=True).stdout
    exported = {ln.split()[-1] for ln in out.splitlines() if " T " in ln}
    assert {"mm_ring_hub_create", "mm_ring_hub_destroy", "mm_ring_create_local"} <= exported


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 3])
def test_c_ring_local_1080p_equals_single_stream(world):
    """mm_ring_step at world 2 and 3 (rank threads on one GPU,
    local transport), 1920x1080, chunk 8, 3 steps with the next step's shift
    posted ahead: per-frame hashes of the whole stream == one rank's stream."""
    n = world * 8 * 3
    common = ["-w", "1920", "-h", "1080", "-n", str(n), "-b", "8", "-l", "5", "-s", "25", "--checksum"]
    a = _checksums(_cli(common, 180))
    b = _checksums(_cli(common + ["--ring-local", str(world)], 240))
    assert len(a) == n and a == b


@pytest.mark.gpu
def test_c_ring_local_c4_world8_2400_frames():
    """C4 itself (BASELINE configs[3]): the 2400-frame 1080p stream frame-
    sharded over 8 ranks in chunks of 300 (rank threads on one GPU, local
    transport), per-frame hashes == the single-rank 2400-frame stream; then
    world 8 with 3 steps of 30-frame chunks (rank 0's carry swap twice, both
    slots reused)."""
    common = ["-w", "1920", "-h", "1080", "-l", "5", "-s", "25", "--checksum"]
    a = _checksums(_cli(common + ["-n", "2400", "-b", "300"], 300))
    b = _checksums(_cli(common + ["-n", "2400", "-b", "300", "--ring-local", "8"], 300))
    assert len(a) == 2400 and a == b
    c = _checksums(_cli(common + ["-n", "720", "-b", "30", "--ring-local", "8"], 240))
    assert c == a[:720]


# ---- round 5: every K2 / band-kernel instance through the ring ----
@pytest.mark.gpu
@pytest.mark.parametrize("name,extra,world,batch,steps", [
    # C3: 3840x2160, L = 6 (the two-band op at N = 4096), batches >= 24 so
    # K2 runs its packed-block and second-half tails, world 3
    ("c3_l6", ["-w", "3840", "-h", "2160", "-l", "6"], 3, 24, 2),
    # standard mode (f1: its own K2 instance and prime), 1080p, world 2
    ("standard", ["-w", "1920", "-h", "1080", "--standard"], 2, 24, 2),
    # steerable O = 8 DIFF (f2: the state is the local-phase planes), world 2
    ("steer_o8_diff", ["-w", "1920", "-h", "1080", "--orientations", "8"], 2, 8, 2),
])
def test_c_ring_local_instances_equal_single_stream(name, extra, world, batch, steps):
    """The prime / in-loop bitwise invariant in every kernel instance the ring
    can carry: rank threads on one GPU (local transport), per-frame FNV-1a
    hashes of the sharded stream == one rank's stream (.cs:142: the only
    temporal state)."""
    n = world * batch * steps
    common = extra + ["-n", str(n), "-b", str(batch), "-s", "25", "--checksum"]
    a = _checksums(_cli(common, 240))
    b = _checksums(_cli(common + ["--ring-local", str(world)], 300))
    assert len(a) == n and a == b


def _compare_summary(txt):
    m = re.search(r"^compare frames (\d+) maxabs (\d+) ndiff (\d+) values (\d+)$", txt, flags=re.M)
    assert m, txt[-2000:]
    per = [(int(t), int(mx), int(nd)) for t, mx, nd in re.findall(r"^cmp (\d+) (\d+) (\d+)$", txt, flags=re.M)]
    return tuple(int(x) for x in m.groups()), per


@pytest.mark.gpu
@pytest.mark.slow
@pytest.mark.timeout(600)
@pytest.mark.parametrize("world,batch,steps", [(2, 300, 2), (3, 300, 1)])
def test_c_ring_local_iir_halo_1080p_o8(world, batch, steps):
    """the IIR steerable filter frame-sharded with a warm-up
    halo (mm_ring_step_halo): each rank restarts its filter from rest
    mm_ring_halo_frames() = 270 frames before its chunk (the slower pole
    (1 - 0.05)^270 < 1e-6).  1080p, O = 8, chunks of 300 frames: the chunks
    not starting within 270 frames of the stream's start differ from the
    single-rank stream, within the RGBA8 parity bar (max 1 LSB on <= 0.1 % of
    values); the first chunk (the stream's own start) is bitwise equal."""
    n = world * batch * steps
    out = _cli(["-w", "1920", "-h", "1080", "--orientations", "8", "--iir", "-n", str(n), "-b", str(batch),
                "-s", "25", "--ring-local", str(world), "--compare"], 540)
    (frames, mx, nd, values), per = _compare_summary(out)
    assert frames == n and len(per) == n
    assert mx <= 1 and nd <= 1e-3 * values, (mx, nd, values)
    for t, fmx, fnd in per:
        if t < batch:   # rank 0 of step 0: the stream's own start, no halo
            assert fnd == 0, (t, fmx, fnd)


def test_ring_step_refuses_iir_without_halo_cpu_args():
    """mm_ring_step_halo validates its arguments before any device work."""
    import ctypes
    L = ctypes.CDLL(LIB)
    L.mm_ring_step_halo.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_int,
                                    ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
    assert L.mm_ring_step_halo(None, 0, None, 0, None, None, None) == -1
    L.mm_ring_halo_frames.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    assert L.mm_ring_halo_frames(None, None) == -1
