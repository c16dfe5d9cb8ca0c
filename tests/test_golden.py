"""Golden fixtures (tests/golden, made by make_golden.py from the CPU oracle and
cross-checked against the float64 twin at generation).

CPU: the fixtures are intact, the synthetic generator still produces their
inputs, and the oracle reproduces their outputs and intermediates.
GPU: the HIP path (C-ABI) matches them within the parity tolerance.
"""
import hashlib
import json
import os

import numpy as np
import pytest

import mmtest as T
import oracle_py as O

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
MAN = json.load(open(os.path.join(GOLD, "manifest.json")))
CASES = sorted(MAN["cases"])


def load(case, key):
    f = MAN["cases"][case]["files"][key]
    a = np.fromfile(os.path.join(GOLD, f["file"]), dtype=f["dtype"]).reshape(f["shape"])
    assert hashlib.sha256(a.tobytes()).hexdigest() == f["sha256"], (case, key)
    return a


def inputs_f32(case):
    return [f.astype(np.float32) / np.float32(255) for f in load(case, "inputs_u8")]


@pytest.mark.parametrize("case", CASES)
def test_generator_reproduces_inputs(case):
    c = MAN["cases"][case]
    ins = load(case, "inputs_u8")
    for t in range(c["frames"]):
        assert np.array_equal(O.synth_frame(c["width"], c["height"], t, gray=c["gray"]), ins[t])


@pytest.mark.parametrize("case", CASES)
def test_oracle_reproduces_outputs(case):
    c = MAN["cases"][case]
    outs = T.oracle_run(c["width"], c["height"], inputs_f32(case), c["levels"], c["phase_scale"],
                        c["edge_mode"], standard=c.get("standard"))
    ref = load(case, "outputs_f32")
    got = np.stack(outs)
    if c["gray"]:
        got = got[..., 0]
    assert np.abs(got - ref).max() <= 1e-6


def test_intermediates_consistent():
    case = "small_L4_S10"
    y = load(case, "f1_y_window")
    F = load(case, "f1_F_centered")
    Fc = O.fft_centered(y)
    assert np.abs(Fc.real - F[..., 0]).max() <= 1e-4 and np.abs(Fc.imag - F[..., 1]).max() <= 1e-4
    A = load(case, "f1_A_centered")
    ymag = O.ifft_mag(A[..., 0] + 1j * A[..., 1])
    assert np.abs(ymag - load(case, "f1_y_mag")).max() <= 1e-6
    assert np.abs(O.blur(ymag) - load(case, "f1_y_blur")).max() <= 1e-6


@pytest.mark.gpu
@pytest.mark.parametrize("case", CASES)
def test_gpu_matches_golden(case):
    c = MAN["cases"][case]
    fr = inputs_f32(case)
    got = np.stack(T.gpu_run(c["width"], c["height"], fr, c["levels"], c["phase_scale"],
                             c["edge_mode"], mode="stream", standard=c.get("standard")))
    ref = load(case, "outputs_f32")
    assert np.array_equal(got[0], fr[0])
    if c["gray"]:
        got = got[..., 0]
    T.assert_close_f32(got[1:], ref[1:], integer_scale=float(c["phase_scale"]).is_integer())


@pytest.mark.gpu
def test_gpu_spectrum_matches_golden():
    import torch
    import mm355
    case = "small_L4_S10"
    c = MAN["cases"][case]
    F = load(case, "f1_F_centered")
    F = F[..., 0] + 1j * F[..., 1]
    h = mm355.Handle(c["width"], c["height"])
    N = h.N
    st = torch.empty(h.state_bytes, dtype=torch.uint8, device="cuda")
    h.compute_state(torch.from_numpy(inputs_f32(case)[1]).cuda(), mm355.RGBA32F, st)
    torch.cuda.synchronize()
    import mmtest as T
    H = c["height"]
    half = T.spectrum_from_state(T.state_rows(st, N, H), N, H)   # the state is G (ABI 8)
    ref = T.centered_to_half(F, N)
    assert np.abs(half - ref).max() / np.abs(ref).max() < 2e-6
    h.close()
