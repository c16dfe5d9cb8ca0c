#!/usr/bin/env python3
"""bench.py — magnified frames/s of the MI355X-native MotionMagnificationProcessor.

Workload (BASELINE.json configs[1]): a synthetic 1920x1080 RGBA8 stream,
5-level pyramid, PhaseScale 25, pyramid mode with orientations = 1 (the
reference's semantics).  One STEP = one mm_process_stream call over the
config's 300-frame stream per GPU (`--frames-per-step`), processed in batches
of 150 frames (`--batch`, mm_set_batch).  Input frames are generated on the
device and resident in HBM before timing.

N > 1 (launched by torch.distributed.run, one rank per GPU): the stream is
frame-sharded: each step rank g processes its own contiguous
chunk and one RCCL ring shift carries the chunk-boundary temporal state
(`--mode ring`, default).  The ring is the C host's (`--ring-impl c`,
default: include/mm_ring.h, lib/libmm_ring.so, its own RCCL communicator;
torch.distributed over gloo only hands rank 0's ring id to the others and
runs the timing barrier and max); `--ring-impl torch` is the Python
ShardedStream over torch.distributed (the gloo rehearsal uses it).
`--mode replicas` runs independent streams (BASELINE configs[4]).  Weak
scaling either way.

Prints ONE JSON line on rank 0 (contract in the task statement) with
`roofline` (dominant kernel, HIP-event time measured on its launch stream
inside the timed region) and `cpu_baseline` (the oracle on host cores, N=1).
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "phase-based-motion-manipulation_amd"))

HBM_PEAK_GBPS = 8000.0          # MI355X HBM3E spec (MI355X_MICROARCH.md)
RESIDENT_BYTES = 32 << 30       # cap on the resident input frames (of 288 GB)


def metric_name(W, H, L, orientations=1, standard=False):
    """BASELINE.json's metric, naming the configuration actually run (the
    default config reproduces BASELINE.json's string exactly)."""
    if standard:
        kind = "standard (non-pyramid) mode"
    elif orientations > 1:
        kind = f"{L}-level {orientations}-orientation steerable pyramid"
    else:
        kind = f"{L}-level pyramid"
    return f"magnified frames/sec at {W}\u00d7{H}, {kind}; achieved HBM GB/s vs peak"


def survey_bytes_per_frame(W, H, N, b_in=4, b_out=4):
    """B = W*H*(2*b_in + b_out) + 6*N^2*8 per output frame
    (dense N x N hand-offs, state read+write every frame)."""
    return W * H * (2 * b_in + b_out) + 6 * N * N * 8


def compulsory_bytes(W, H, N, frames, b_in=4, b_out=4):
    """Per-launch algorithmic bytes of each kernel in this design: every input
    and output byte it must move, once.  F = N/2+1 half-spectrum
    columns, Hn = H+4 rows kept for the crop + vertical blur."""
    F, Hn = N // 2 + 1, min(H + 4, N)
    Hq = Hn + (Hn & 1)
    # k_cols: every frame's G in and Q out, plus the state G_{t-1} (the
    # previous frame's row spectra, F x H) read once per launch (ABI 8; the
    # state is no longer a 2D spectrum stored and reloaded)
    return {"k_rows_fwd": frames * (W * H * b_in + F * H * 8),
            "k_cols": frames * (F * H * 8 + F * Hq * 8) + F * H * 8,
            "k_rows_inv": frames * (F * Hq * 8 + Hn * W * 4),
            "k_compose": frames * (Hn * W * 4 + W * H * (b_in + b_out)),
            # K3 + K4 fused (even sizes): Q once, the input for I/Q, the output
            "k_rows_inv_compose": frames * (F * Hq * 8 + W * H * (b_in + b_out))}


def steer_bytes_per_frame(W, H, N, L, O, iir, minf=0.05, maxf=0.45, b_in=4, b_out=4):
    """Compulsory bytes per frame of the steerable extension's kernels (f2,
    csrc/mm_steer.hpp), by profiling id (mm_profile_end): k_rows_fwd (K1: frame
    in, G out), k_cols (k_cols_fwd: G in, half spectrum Fb out; k_sb_cols: Fb
    in, the band rows T out for the columns each band is nonzero in), k_rows_inv
    (k_sb_rows: T in, the local-phase state planes in and out, Yh out),
    k_compose (Yh and the frame in, the output frame out).  Band b of middle
    level i is identically zero in column kx when |kx/N| > hi_i (band_col_zero),
    so only the other columns' rows are moved."""
    F, Hn = N // 2 + 1, min(H + 4, N)
    Hq = Hn + (Hn & 1)
    Wc = W + 4
    nmid = L - 2 if L >= 3 else 0
    nb = nmid * (O // 2)
    cols = []
    for i in range(1, L - 1):                       # build_spec (mm_api.hip)
        r = float("nan") if L == 3 else (i - 1) / (L - 3)
        c = minf * (maxf / minf) ** (1.0 - r)
        hi = 1.5 * c
        n = sum(1 for k in range(N) if not (abs((k if k < N // 2 else k - N) / N) > hi))
        cols.append(n)
    t_rows = sum(cols[b % nmid] for b in range(nb)) if nmid else 0
    t_rows += N                                      # the residual band: every column
    T_bytes = t_rows * Hq * 8
    planes = 3 if iir else 1
    state = nb * Hn * Wc * 4 * planes
    return {"k_rows_fwd": W * H * b_in + F * H * 8,
            "k_cols": F * H * 8 + F * N * 8 + F * N * 8 + T_bytes,
            "k_rows_inv": T_bytes + 2 * state + Hn * W * 4,
            "k_compose": Hn * W * 4 + W * H * (b_in + b_out)}


def profile_key(W, H, L, orientations, standard, filt):
    """The configuration a committed profile (profiles/traffic.json,
    profiles/valu.json: their "config" entry) was measured on; bench lines
    quote PMC traffic and VALU figures only for that configuration."""
    mode = "standard" if standard else (f"steer{orientations}{filt}" if orientations > 1 else "pyramid")
    return f"{W}x{H}_L{L}_{mode}"


def load_profile(name, key):
    """profiles/NAME (the default configuration's) or profiles/<stem>_<key>.json,
    whichever records `key` as its measured configuration; else None."""
    stem = name[:-5] if name.endswith(".json") else name
    for fn in (f"{stem}_{key}.json", name):
        try:
            d = json.load(open(os.path.join(ROOT, "profiles", fn)))
        except Exception:
            continue
        if d.get("config") == key:
            return d
    return None


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--frames-per-step", type=int, default=300,
                    help="frames per step and GPU: one mm_process_stream call over the "
                         "config's 300-frame stream by default")
    ap.add_argument("--batch", type=int, default=150,
                    help="frames per K1/K2/K3/K4 batch inside a step (mm_set_batch; 0: the "
                         "whole step)")
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--levels", type=int, default=5)
    ap.add_argument("--phase-scale", type=float, default=25.0)
    ap.add_argument("--mode", choices=("ring", "replicas"), default="ring")
    ap.add_argument("--standard", action="store_true",
                    help="usePyramidDecomposition=false (standard mode, SURVEY f1)")
    ap.add_argument("--orientations", type=int, default=1,
                    help=">1: MM_MODE_STEERABLE extension (SURVEY f2; BASELINE's "
                         "'8-orientation' wording), 4/6/8 oriented subbands per level")
    ap.add_argument("--temporal-filter", choices=("diff", "iir"), default="diff",
                    help="steerable extension's temporal filter (iir: no ring mode)")
    ap.add_argument("--dist-backend", choices=("nccl", "gloo"), default="nccl",
                    help="gloo: rehearsal of the N>1 path without RCCL (ranks may share one "
                         "GPU; the ring state goes through host memory; implies --ring-impl torch)")
    ap.add_argument("--ring-impl", choices=("c", "torch"), default="c",
                    help="--mode ring transport: c = the C host's RCCL ring (libmm_ring.so, "
                         "mm_ring_step per step); torch = mm355.ShardedStream over torch.distributed")
    ap.add_argument("--ring-self", action="store_true",
                    help="rehearsal at world 1: run the C ring anyway (RCCL send/recv to itself "
                         "every step)")
    ap.add_argument("--checksum", action="store_true",
                    help="rehearsal: print per-frame output checksums (all ranks, rank 0) "
                         "instead of the bench line; sharded and single-rank runs of the "
                         "same frames must agree bitwise")
    ap.add_argument("--replica-index", type=int, default=None,
                    help="--mode replicas: which replica's stream this process runs "
                         "(default: its RANK; seed = base + index)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=15.0,
                    help="bound on the CPU-baseline sample")
    ap.add_argument("--call-pattern", choices=("batch", "per-frame"), default="batch",
                    help="per-frame: the reference's own call pattern (OnRenderImage once "
                         "per frame, .cs:101-143): mm_process on device pointers, one frame "
                         "per call, batch size 1 (N=1 only)")
    ap.add_argument("--drop-in-frames", type=int, default=300,
                    help="frames of the per-frame drop-in leg reported beside the batch "
                         "rate (0: skip)")
    # internal: CPU-baseline child process (cpu_baseline)
    ap.add_argument("--cpu-worker", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--cpu-out", help=argparse.SUPPRESS)
    ap.add_argument("--cpu-threads", type=int, default=1, help=argparse.SUPPRESS)
    ap.add_argument("--cpu-frames", type=int, default=30, help=argparse.SUPPRESS)
    ap.add_argument("--cpu-keep", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--cpu-pairs", default="", help=argparse.SUPPRESS)
    return ap.parse_args(argv)


def parse_args(argv):
    return parse(argv)


class GpuBackend:
    """ShardedStream backend over one mm355 handle; frames pre-generated."""

    def __init__(self, handle, frames, out, fmt, chunk, world, rank, torch, host_exchange=False,
                 per_frame=False):
        self.h, self.frames, self.out, self.fmt = handle, frames, out, fmt
        self.per_frame = per_frame    # --call-pattern per-frame: one mm_process per frame
        self.chunk, self.world, self.rank, self.torch = chunk, world, rank, torch
        self.host = host_exchange     # gloo rehearsal: exchanged states live on the host
        self.sums = None              # --checksum: global frame index -> byte sum

    def _stream(self):
        return self.torch.cuda.current_stream().cuda_stream

    def _local(self, frame_index):
        step = frame_index // (self.world * self.chunk)
        return step, frame_index - step * self.world * self.chunk - self.rank * self.chunk

    def empty_state(self):
        return self.torch.empty(self.h.state_bytes, dtype=self.torch.uint8,
                                device="cpu" if self.host else "cuda")

    def state_of(self, frame_index):
        s, k = self._local(frame_index)
        buf = self.torch.empty(self.h.state_bytes, dtype=self.torch.uint8, device="cuda")
        self.h.compute_state(self.frames[s % len(self.frames), k], self.fmt, buf,
                             stream=self._stream())
        return buf.cpu() if self.host else buf

    def set_state(self, buf):
        if self.host:
            buf = buf.cuda()
        self.h.set_state(buf, stream=self._stream())

    def reset(self):
        self.h.reset()

    def process(self, lo, count):
        s, k = self._local(lo)
        if self.per_frame:
            src = self.frames[s % len(self.frames)]
            for i in range(count):
                self.h.process(src[k + i], self.out[i], self.fmt, on_device=True,
                               stream=self._stream())
        else:
            self.h.process_stream(self.frames[s % len(self.frames), k], self.out, count, self.fmt,
                                  stream=self._stream())
        if self.sums is not None:
            v = self.out[:count].reshape(count, -1).sum(dim=1, dtype=self.torch.int64).cpu()
            for i in range(count):
                self.sums[lo + i] = int(v[i])


def _cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def available_cpus():
    """CPUs this process may run on: the affinity mask, capped by a cgroup v2
    CPU quota when one is set (a GPU box shows every host CPU in
    os.cpu_count() but grants each job a share)."""
    try:
        n = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        n = os.cpu_count() or 1
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            n = min(n, max(1, -(-int(q) // int(per))))
    except (OSError, ValueError):
        pass
    return n


def _cpu_worker(a):
    """Child process of cpu_baseline: times the oracle on `--cpu-threads`
    threads (bound by OMP_PROC_BIND/OMP_PLACES from the parent's env, read when
    libgomp loads) and writes its record (+ RGBA8 outputs) to --cpu-out."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import numpy as np
    import oracle_py as O
    W, H, L, S = a.width, a.height, a.levels, a.phase_scale
    thr = O.set_threads(a.cpu_threads)
    o = O.Oracle(W, H, levels=L, phase_scale=S)
    if a.standard:
        o.set_standard(True)
    outs = [o.process(O.synth_frame(W, H, 0))]    # passthrough, not timed
    n, t0 = 0, time.perf_counter()
    while n < a.cpu_frames:
        y = o.process(O.synth_frame(W, H, n + 1))
        if a.cpu_keep:
            outs.append(y)
        n += 1
        if time.perf_counter() - t0 >= a.cpu_seconds:
            break
    dt = time.perf_counter() - t0
    pairs = [int(t) for t in a.cpu_pairs.split(",")] if a.cpu_pairs else []
    if pairs:
        # untimed: the output of frame t needs only frames t-1 and t (.cs:142),
        # so the launch-boundary frames of the timed step come from a reset
        # oracle fed those two frames
        po = []
        for t in pairs:
            o.reset()
            o.process(O.synth_frame(W, H, t - 1))
            po.append(o.process(O.synth_frame(W, H, t)))
        np.save(a.cpu_out + ".pairs.npy", np.stack(po))
    o.close()
    if a.cpu_keep:
        np.save(a.cpu_out + ".npy", np.stack(outs))
    json.dump({"threads": thr, "frames": n, "seconds": dt}, open(a.cpu_out, "w"))


def cpu_baseline(a):
    """The CPU oracle (literal restatement of the reference algorithm: radix-2,
    2 forward FFTs per frame, per-level passes) on a bounded sample of the same
    stream, all-core (every CPU available to this job, threads bound with
    OMP_PROC_BIND=close / OMP_PLACES=cores) and single-thread, each in its own
    process so the OpenMP binding applies.  Returns (record, outputs): the
    all-core run's RGBA8 frames 0..n feed the parity check."""
    import subprocess
    import tempfile
    import numpy as np
    W, H, L, S = a.width, a.height, a.levels, a.phase_scale
    cores = available_cpus()

    def run(threads, max_frames, seconds, keep, pairs=()):
        with tempfile.TemporaryDirectory() as d:
            out = os.path.join(d, "cpu.json")
            env = dict(os.environ, OMP_NUM_THREADS=str(threads), OMP_PROC_BIND="close",
                       OMP_PLACES="cores")
            cmd = [sys.executable, os.path.abspath(__file__), "--cpu-worker", "--cpu-out", out,
                   "--cpu-threads", str(threads), "--cpu-frames", str(max_frames),
                   "--cpu-seconds", str(seconds), "--width", str(W), "--height", str(H),
                   "--levels", str(L), "--phase-scale", str(S)]
            if keep:
                cmd.append("--cpu-keep")
            if pairs:
                cmd += ["--cpu-pairs", ",".join(str(t) for t in pairs)]
            if a.standard:
                cmd.append("--standard")
            subprocess.run(cmd, env=env, check=True, timeout=seconds * 4 + 240)
            rec = json.load(open(out))
            outs = np.load(out + ".npy") if keep else None
            pouts = np.load(out + ".pairs.npy") if pairs else None
        return rec["threads"], rec["frames"], rec["seconds"], outs, pouts

    pairs = boundary_frames(a.frames_per_step, min(a.batch or a.frames_per_step, a.frames_per_step),
                            W, H)
    thr, n, dt, outs, pouts = run(cores, 30, a.cpu_seconds, True, pairs)
    _, n1, dt1, _, _ = run(1, 30, a.cpu_seconds / 3, False)
    rec = {"value": round(n / dt, 4), "unit": "frames/s", "cores": thr, "kind": "port",
           "single_thread_value": round(n1 / dt1, 4), "single_thread_frames": n1,
           "cpu_model": _cpu_model(), "host_cpus": os.cpu_count(), "cpus_available": cores,
           "binding": "OMP_PROC_BIND=close OMP_PLACES=cores",
           "sample": f"{n} frames (t=1..{n}) of the same {W}x{H} synthetic RGBA8 stream "
                     f"(seed 0x5EED0000), L={L}, S={S}, after the passthrough frame; literal "
                     f"fp32 C restatement (radix-2, 2 forward FFTs/frame, per-level passes), "
                     f"OpenMP {thr} threads (every CPU available to this job: affinity mask "
                     f"and cgroup quota; the host shows {os.cpu_count()}); single-thread on "
                     f"t=1..{n1}"}
    return rec, (outs, pairs, pouts)


def boundary_frames(C, B, W, H):
    """The frames of a C-frame step in batches of B where K2's launch shape
    changes (mm_api.hip launch_k2): each batch's first frames (the prime from
    the state slot), the packed block's hand-off to k_cols_tail (40 % of the
    batch at N <= 2048, 30 % at N = 4096), the second-half blocks' tails (10 %)
    and each batch's last frame.  Frames 1..30 are checked in sequence anyway."""
    N = 1
    while N < max(W, H):
        N *= 2
    tail_pct = 30 if N >= 4096 else 40
    out = set()
    for b in range(0, C, B):
        nf = min(B, C - b)
        k = max(0, min(nf * tail_pct // 100, nf - 2)) if nf >= 24 else 0
        k2t = min(nf * 10 // 100, nf - 2) if nf >= 24 else 0
        for t in (b, b + 1, b + nf - k - 1, b + nf - k, b + nf - k2t - 1, b + nf - k2t, b + nf - 1):
            if 31 <= t < C:
                out.add(t)
    return sorted(out)


def parity_check(mm355, torch, params, W, H, ref, local, C, B):
    """The timed step itself against the oracle: a fresh handle at the timed
    batch B processes the step's C frames (one mm_process_stream call, the
    same launch shapes as the timed region: K2's prime, packed-block and
    second-half tails), and its output frames 0..n (the oracle's sequential
    run in cpu_baseline) and every launch-boundary frame (boundary_frames:
    the oracle fed frames t-1, t) are held to SURVEY.md §8c's RGBA8 bar:
    exact except +-1 LSB on <= 0.1% of values; frame 0 bitwise."""
    import numpy as np
    seq, pairs, pref = ref
    n = seq.shape[0]
    h = mm355.Handle(W, H, params, device=local)
    h.set_batch(B)
    fr = torch.empty((C, H, W, 4), dtype=torch.uint8, device="cuda")
    out = torch.empty_like(fr)
    st = torch.cuda.current_stream().cuda_stream
    h.synth(fr, 0, C, seed=0x5EED0000, stream=st)
    h.process_stream(fr, out, C, mm355.RGBA8, stream=st)
    torch.cuda.synchronize()
    idx = list(range(n)) + list(pairs)
    got = out[idx].cpu().numpy()
    h.close()
    want = np.concatenate([seq, pref]) if len(pairs) else seq
    d = np.abs(got.astype(np.int16) - want.astype(np.int16))
    return {"frames": len(idx), "sequence": f"0..{n - 1}", "boundary_frames": list(pairs),
            "launch_shape": f"{C} frames in one call, batches of {B} (the timed step)",
            "first_frame_bitwise": bool(np.array_equal(got[0], seq[0])),
            "max_abs_lsb": int(d.max()), "frac_values_off": float((d > 0).mean()),
            "rmse_lsb": round(float(np.sqrt((d.astype(np.float64) ** 2).mean())), 5),
            "bar": "max 1 LSB, <= 0.1% of values"}


class _DevEvents:
    """HIP events with a device-scope release (hipEventDisableSystemFence):
    torch.cuda.Event records with a system-scope fence, a cache write-back per
    record that would lengthen the one-frame calls it brackets."""
    FLAGS = 0x20000000   # hipEventDisableSystemFence (hip_runtime_api.h)

    def __init__(self, n):
        import ctypes
        self.ct = ctypes
        self.hip = ctypes.CDLL("libamdhip64.so.7")   # the runtime torch and libmm355 share
        self.ev = []
        for _ in range(n):
            e = ctypes.c_void_p()
            assert self.hip.hipEventCreateWithFlags(ctypes.byref(e), ctypes.c_uint(self.FLAGS)) == 0
            self.ev.append(e)

    def record(self, k, stream):
        assert self.hip.hipEventRecord(self.ev[k], self.ct.c_void_p(stream)) == 0

    def elapsed_ms(self, a, b):
        ms = self.ct.c_float()
        assert self.hip.hipEventElapsedTime(self.ct.byref(ms), self.ev[a], self.ev[b]) == 0
        return ms.value

    def close(self):
        for e in self.ev:
            self.hip.hipEventDestroy(e)


def drop_in_per_frame(mm355, torch, params, W, H, frames, local, count):
    """The reference's call pattern (OnRenderImage once per frame,
    .cs:101-143): a fresh handle at batch size 1, mm_process with device
    pointers, one frame per call on one stream.  Every call re-transforms the
    state G_{t-1} (K2's priming column FFT of the previous frame's row
    spectra) and makes one launch per kernel.  frames/s: the calls alone
    (wall clock, after the passthrough frame and 10 warm-up calls); latency:
    a second pass with device-scope HIP events around each call."""
    h = mm355.Handle(W, H, params, device=local)
    h.set_batch(1)
    src = frames.reshape(-1, H, W, 4)
    out = torch.empty((2, H, W, 4), dtype=torch.uint8, device="cuda")
    st = torch.cuda.current_stream()
    sp = st.cuda_stream
    warm = 11
    count = min(count, src.shape[0] - warm)
    for k in range(warm):
        h.process(src[k], out[k & 1], mm355.RGBA8, on_device=True, stream=sp)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(count):
        h.process(src[warm + k], out[k & 1], mm355.RGBA8, on_device=True, stream=sp)
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    ev = _DevEvents(count + 1)
    ev.record(0, sp)
    for k in range(count):
        h.process(src[warm + k], out[k & 1], mm355.RGBA8, on_device=True, stream=sp)
        ev.record(k + 1, sp)
    torch.cuda.synchronize()
    lat = sorted(ev.elapsed_ms(k, k + 1) for k in range(count))
    ev.close()
    h.close()
    pick = lambda q: round(lat[min(count - 1, int(q * count))], 5)
    return {"frames": count, "frames_per_s": round(count / wall, 2),
            "latency_ms": {"mean": round(sum(lat) / count, 5), "p50": pick(0.5),
                           "p99": pick(0.99), "max": round(lat[-1], 5)},
            "pattern": "mm_process(MM_FRAMES_ON_DEVICE), batch 1, one call per frame "
                       "(.cs:101-143 OnRenderImage); frames/s = calls / wall time; latency = "
                       "device-scope HIP events around each call on its stream (second pass)"}


def frame_roofline(W, H, N, fps_per_gpu, batch, dom_traffic=None, ran=None, key=None, per_frame_bytes=None):
    """Frame-level HBM roofline: the design's compulsory bytes per output
    frame (compulsory_bytes() of the kernels that ran, at this batch size, per
    frame) x frames/s per GPU vs 8 TB/s; PMC bytes per frame
    (profiles/traffic.json, rocprofv3 FETCH_SIZE/WRITE_SIZE) beside them."""
    if per_frame_bytes is not None:    # steerable: bytes per frame by kernel
        cb = {k: v * batch for k, v in per_frame_bytes.items()}
    else:
        cb = compulsory_bytes(W, H, N, batch)
    if ran is None:
        ran = [k for k in cb if k != "k_rows_inv_compose"]
    per_frame = sum(cb[k] for k in ran if k in cb) / batch
    rec = {"bytes_per_frame": int(per_frame),
           "achieved_GBps": round(per_frame * fps_per_gpu / 1e9, 1),
           "peak": HBM_PEAK_GBPS, "frac": round(per_frame * fps_per_gpu / 1e9 / HBM_PEAK_GBPS, 4),
           "pmc_bytes_per_frame": None, "pmc_ratio": None,
           "note": "compulsory bytes per frame of the kernels that ran (" + "+".join(ran) +
                   "; DESIGN.md §5) x frames/s per GPU"}
    tj = load_profile("traffic.json", key)
    if tj is not None:
        try:
            pmc = sum(tj["kernels"][k]["hbm_bytes_per_frame"] for k in ran)
            rec["pmc_bytes_per_frame"] = int(pmc)
            rec["pmc_ratio"] = round(pmc / per_frame, 4)
            rec["pmc_source"] = "profiles/traffic.json"
        except Exception:
            pass
    return rec


def main():
    a = parse()
    if a.cpu_worker:
        return _cpu_worker(a)
    import torch
    import torch.distributed as dist
    import mm355
    from mm355.stream import ShardedStream

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != a.gpus and rank == 0:
        print(f"warning: --gpus {a.gpus} but WORLD_SIZE {world}", file=sys.stderr)
    gloo = a.dist_backend == "gloo"
    # the C ring carries the data path over its own RCCL communicator; the
    # process group only exchanges the ring id, the barrier and the max time
    c_ring = a.mode == "ring" and not gloo and a.ring_impl == "c" and (world > 1 or a.ring_self)
    # gloo rehearsal: ranks may share the box's GPU(s)
    dev = local % torch.cuda.device_count() if gloo else local
    torch.cuda.set_device(dev)
    if world > 1:
        if gloo or c_ring:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", dev))
    W, H, C = a.width, a.height, a.frames_per_step
    steer = a.orientations > 1
    if steer and a.temporal_filter == "iir" and a.mode == "ring" and world > 1:
        # the IIR state is a history of frames: mm_compute_state refuses it
        raise SystemExit("--temporal-filter iir cannot be frame-sharded: use --mode replicas")
    if steer:
        params = mm355.Params.make(levels=a.levels, phase_scale=a.phase_scale,
                                   mode=mm355.MODE_STEERABLE, orientations=a.orientations,
                                   temporal_filter=1 if a.temporal_filter == "iir" else 0)
    else:
        params = mm355.Params.make(levels=a.levels, phase_scale=a.phase_scale,
                                   mode=mm355.MODE_STANDARD if a.standard else mm355.MODE_PYRAMID)
    h = mm355.Handle(W, H, params, device=dev)
    per_frame = a.call_pattern == "per-frame"
    # one step = one batch: K2 keeps F_{t-1} on chip across it; the per-frame
    # pattern is the reference's one OnRenderImage per frame (batch 1)
    B = 1 if per_frame else min(a.batch or C, C)
    h.set_batch(B)
    N = h.N

    # resident inputs: one buffer per step (warmup + timed), generated on
    # device, at most RESIDENT_BYTES of them (4K x 25 steps would take 249 GB
    # of the 288 GB): step s then reads buffer s mod nbuf, which holds
    # frames of an earlier step; every step still moves all of its bytes
    total_steps = a.warmup + a.steps
    ring = a.mode == "ring" and world > 1 and not c_ring
    replica = rank if a.replica_index is None else a.replica_index
    seed = 0x5EED0000 + (0 if a.mode == "ring" else replica)
    step_bytes = C * H * W * 4
    nbuf = max(2, min(total_steps, RESIDENT_BYTES // step_bytes))
    frames = torch.empty((nbuf, C, H, W, 4), dtype=torch.uint8, device="cuda")
    for s in range(nbuf):
        t0 = (s * world * C + rank * C) if a.mode == "ring" else s * C
        h.synth(frames[s], t0, C, seed=seed, stream=torch.cuda.current_stream().cuda_stream)
    out = torch.empty((C, H, W, 4), dtype=torch.uint8, device="cuda")
    backend = GpuBackend(h, frames, out, mm355.RGBA8, C, world if ring else 1,
                         rank if ring else 0, torch, host_exchange=gloo, per_frame=per_frame)
    stream = ShardedStream(backend, C, rank if ring else 0, world if ring else 1)
    if a.checksum:
        backend.sums = {}
    cring = None
    if c_ring:
        if per_frame:
            raise SystemExit("--call-pattern per-frame is a single-GPU measurement")
        rid = [mm355.new_ring_id() if rank == 0 else None]
        if world > 1:
            dist.broadcast_object_list(rid, src=0)
        cring = mm355.Ring(world, rank, rid[0], dev, h, C, mm355.RGBA8)
    torch.cuda.synchronize()

    # ring mode overlaps each step's state shift with the previous step's
    # compute (ShardedStream prefetch / mm_ring_step's next_last); the shift
    # for a step past the end is never posted
    def run_step(s):
        if cring is None:
            stream.step(s, prefetch=ring and s + 1 < total_steps)
            return
        nxt = frames[(s + 1) % nbuf, C - 1] if s + 1 < total_steps else None
        cring.step(s, frames[s % nbuf], out, nxt, stream=torch.cuda.current_stream().cuda_stream)
        if backend.sums is not None:
            v = out.reshape(C, -1).sum(dim=1, dtype=torch.int64).cpu()
            lo = s * world * C + rank * C
            for i in range(C):
                backend.sums[lo + i] = int(v[i])

    for s in range(a.warmup):
        run_step(s)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    h.profile_begin()
    t_start = time.perf_counter()
    for s in range(a.warmup, total_steps):
        run_step(s)
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t_start
    prof = h.profile_end()
    stream.finish()
    if cring is not None:
        cring.close()   # retires shifts posted ahead
    if a.checksum:
        sums = backend.sums
        if world > 1 and a.mode == "ring":   # (gloo or nccl process group)
            allv = [None] * world
            dist.all_gather_object(allv, sums)
            sums = {k: v for d in allv for k, v in d.items()}
        if a.mode == "replicas":   # every rank's own stream, keyed by rank
            mine = [sums[k] for k in sorted(sums)]
            allv = [None] * world
            if world > 1:
                dist.all_gather_object(allv, mine)
            else:
                allv = [mine]
            if rank == 0:
                print(json.dumps({"checksums_by_rank": {str(r): v for r, v in enumerate(allv)},
                                  "world": world, "inputs_wrapped": nbuf < total_steps}), flush=True)
        elif rank == 0:
            # inputs_wrapped: the resident buffers repeat (step s reads s mod nbuf),
            # so the sums are not those of the single-rank stream of that length
            # and a ring-vs-single comparison must not trust them
            print(json.dumps({"checksums": [sums[k] for k in sorted(sums)],
                              "frames": sorted(sums)[:1] + sorted(sums)[-1:], "world": world,
                              "inputs_wrapped": nbuf < total_steps}),
                  flush=True)
        if world > 1:
            dist.destroy_process_group()
        return
    if world > 1:
        dist.barrier()
        t = torch.tensor([elapsed], dtype=torch.float64, device="cpu" if gloo or c_ring else "cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    frames_total = a.steps * C * world
    fps = frames_total / elapsed
    key = profile_key(W, H, a.levels, a.orientations, a.standard, a.temporal_filter)
    sbytes = (steer_bytes_per_frame(W, H, N, a.levels, a.orientations, a.temporal_filter == "iir")
              if steer else None)
    kern = {}
    for name, (ms, launches, nfr) in prof.items():
        if launches:
            if steer:   # bytes per frame x frames over the kernel's summed time
                ab = round(sbytes[name] * nfr / launches) if name in sbytes else None
            else:
                ab = compulsory_bytes(W, H, N, nfr // launches).get(name)
            kern[name] = {"ms_total": round(ms, 4), "launches": launches, "frames": nfr,
                          "us_per_frame": round(ms * 1e3 / nfr, 3),
                          "ms_per_launch": round(ms / launches, 5),
                          "algorithmic_bytes_per_launch": ab,
                          "achieved_GBps": (round(ab / (ms / launches * 1e-3) / 1e9, 1)
                                            if ab else None)}
    dom = max(kern, key=lambda k: kern[k]["ms_total"])
    dk = kern[dom]
    achieved = dk["achieved_GBps"]
    traffic = None
    tj = load_profile("traffic.json", key)
    if tj is not None:
        try:
            pmc_frame = tj["kernels"][dom]["hbm_bytes_per_frame"]
            traffic = round(pmc_frame * dk["frames"] / dk["launches"])
        except Exception:
            traffic = None
    valu = None
    vj_all = load_profile("valu.json", key)
    if vj_all is not None:
        try:
            vj = vj_all[dom]
            valu = {"valu_busy": vj["valu_busy"], "valu_insts_per_launch": vj["valu_insts_per_launch"],
                    "source": "profiles/valu.json: rocprofv3 SQ_INSTS_VALU x 4 cycles (measured "
                              "issue cost of a wave64 VALU instruction, "
                              "profiles/r02_valu_calib.json) / (1024 SIMDs x kernel cycles)"}
        except Exception:
            valu = None
    B_survey = survey_bytes_per_frame(W, H, N)
    batch = B

    result = {
        "metric": metric_name(W, H, a.levels, a.orientations, a.standard), "value": round(fps, 2), "unit": "frames/s", "n_gpus": world,
        "steps": a.steps, "warmup": a.warmup, "ms_per_step": round(elapsed * 1e3 / a.steps, 4),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f32",
        "data": "synthetic",
        "config": {"workload": (f"{W}x{H} RGBA8 synthetic stream, {a.levels}-level steerable "
                                f"extension, {a.orientations} orientations, {a.temporal_filter} "
                                f"temporal filter, PhaseScale={a.phase_scale}" if steer else
                                f"{W}x{H} RGBA8 synthetic stream, standard (non-pyramid) mode, "
                                f"PhaseScale={a.phase_scale}" if a.standard else
                                f"{W}x{H} RGBA8 synthetic stream, {a.levels}-level pyramid, "
                                f"PhaseScale={a.phase_scale}, orientations=1 (reference semantics)"),
                   "frames_per_step_per_gpu": C, "padded_n": N,
                   # step s reads resident buffer s mod nbuf: past nbuf steps the
                   # synthetic stream repeats (every step still moves its bytes)
                   "inputs_wrapped": nbuf < total_steps,
                   "call_pattern": ("one mm_process per frame (batch 1)" if per_frame else
                                    f"mm_process_stream, {C} frames per call in batches of {B}"),
                   "parallelism": ("single GPU" if world == 1 and not c_ring else
                                   f"frame-sharded x{world}, C host RCCL ring (libmm_ring "
                                   f"mm_ring_step, state {h.state_bytes} B per hop)" if c_ring else
                                   f"frame-sharded x{world}, "
                                   + ("gloo rehearsal, ring state via host" if gloo
                                      else "torch.distributed RCCL ring state shift")
                                   if ring else f"replicas x{world}")},
        "roofline": {"bound": "hbm", "kernel": dom, "achieved": achieved,
                     "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBPS, 5) if achieved else None,
                     "traffic": traffic,
                     "bytes_model": "compulsory bytes of the dominant kernel (DESIGN.md §5); "
                                    "traffic = rocprofv3 FETCH_SIZE*2+WRITE_SIZE per launch "
                                    "(profiles/traffic.json, quoted only when measured on this "
                                    "configuration: " + key + ")",
                     "compute": valu},
        "frame_roofline": frame_roofline(W, H, N, fps / world, batch, ran=list(kern), key=key,
                                         per_frame_bytes=sbytes),
        "survey_model": {"bytes_per_frame": B_survey,
                         "equivalent_GBps_per_gpu": round(B_survey * fps / world / 1e9, 1),
                         "note": "SURVEY.md §8(d) B=W*H*(2b_in+b_out)+6*N^2*8 charges dense "
                                 "N x N hand-offs and a per-frame state round trip that this "
                                 "design does not move; B x fps is an equivalent rate, not a "
                                 "roofline fraction (it can exceed peak). The frame-level "
                                 "fraction is frame_roofline.frac"},
        "kernels": kern,
    }
    h.close()
    if world == 1 and not per_frame and a.drop_in_frames > 0 and not steer and not a.checksum:
        # the reference's call pattern beside the batch rate (same frames)
        result["drop_in_per_frame"] = drop_in_per_frame(mm355, torch, params, W, H, frames,
                                                        local, a.drop_in_frames)
    if rank == 0 and world == 1 and not a.no_cpu_baseline and not steer:
        result["cpu_baseline"], ref = cpu_baseline(a)
        result["parity_vs_oracle"] = parity_check(mm355, torch, params, W, H, ref, local, C, B)
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
