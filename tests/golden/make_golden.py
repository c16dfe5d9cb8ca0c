#!/usr/bin/env python3
"""Generate the committed golden fixtures (tests/golden/*.bin + manifest.json).

Produced by the CPU oracle (oracle/mm_ref.c, the literal fp32 restatement of
the reference pipeline) and cross-checked at generation time against the
independent float64 numpy twin (tests/np_twin.py): generation aborts if they
disagree beyond 5e-6.  The reference itself (Unity C#/HLSL) cannot run here and
ships no vectors, so these fixtures pin the GPU path to the
oracle, not to reference-produced outputs.

Raw little-endian arrays; shapes/dtypes/params in manifest.json.
"""
import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
import np_twin  # noqa: E402
import oracle_py as O  # noqa: E402

CASES = [
    # name, W, H, levels, phase_scale, edge, gray, frames, dump intermediates
    ("small_L4_S10", 64, 48, 4, 10.0, 0, False, 4, True),
    ("small_L5_S9p7", 64, 48, 5, 9.7, 0, False, 4, False),
    ("small_L6_S25_clamp", 64, 48, 6, 25.0, 1, False, 4, False),
    ("wide_L5_S25", 200, 120, 5, 25.0, 0, False, 3, False),
    ("c1_256_gray_L3_S10", 256, 256, 3, 10.0, 0, True, 4, False),
]
# standard (non-pyramid) mode cases (f1): name -> oracle set_standard() kwargs
STANDARD = {"std_96x64_S25": (96, 64, 5, 25.0, 0, False, 3, False, {}),
            "std_64x48_S9p7_steep2": (64, 48, 5, 9.7, 1, False, 3, False,
                                       {"steep": 2.0, "high": 0.3})}


def save(name, arr, manifest, entry):
    fn = f"{name}.bin"
    arr = np.ascontiguousarray(arr)
    arr.tofile(os.path.join(HERE, fn))
    entry.setdefault("files", {})[name.split("__")[-1]] = {
        "file": fn, "dtype": str(arr.dtype), "shape": list(arr.shape),
        "sha256": hashlib.sha256(arr.tobytes()).hexdigest()}


def main():
    O.build()
    manifest = {"generator": "tests/golden/make_golden.py (CPU oracle, fp32)",
                "seed": 0x5EED0000, "min_freq": 0.05, "max_freq": 0.45,
                "magnitude_threshold": 0.01, "cases": {}}
    cases = [c + (None,) for c in CASES] + [(k,) + v for k, v in STANDARD.items()]
    for name, W, H, L, S, edge, gray, nf, dump, std in cases:
        frames = [O.synth_frame(W, H, t, gray=gray) for t in range(nf)]
        ff = [f.astype(np.float32) / np.float32(255) for f in frames]
        o = O.Oracle(W, H, levels=L, phase_scale=S, edge_mode=edge)
        if std is not None:
            o.set_standard(True, **std)
        outs, dbg = [], None
        for k, f in enumerate(ff):
            if dump and k == 1:
                out, dbg = o.process(f, dbg=True)
            else:
                out = o.process(f)
            outs.append(out)
        for k in range(1, nf):
            tw = np_twin.process_frame(ff[k].astype(np.float64), ff[k - 1].astype(np.float64),
                                       L, 0.05, 0.45, S, edge=edge, standard=std)
            err = float(np.abs(outs[k] - tw).max())
            assert err < 5e-6, (name, k, err)
        entry = {"width": W, "height": H, "levels": L, "phase_scale": S, "edge_mode": edge,
                 "gray": gray, "frames": nf}
        if std is not None:
            entry["standard"] = std
        save(f"{name}__inputs_u8", np.stack(frames), manifest, entry)
        out = np.stack(outs)
        if gray:   # R = G = B (to fp32 rounding), alpha = 1: keep R only
            out = out[..., 0]
        save(f"{name}__outputs_f32", out, manifest, entry)
        if dbg is not None:
            save(f"{name}__f1_y_window", dbg["y_cur"], manifest, entry)
            save(f"{name}__f1_F_centered", np.stack([dbg["F_cur"].real, dbg["F_cur"].imag], -1)
                 .astype(np.float32), manifest, entry)
            save(f"{name}__f1_A_centered", np.stack([dbg["A"].real, dbg["A"].imag], -1)
                 .astype(np.float32), manifest, entry)
            save(f"{name}__f1_y_mag", dbg["y_mag"], manifest, entry)
            save(f"{name}__f1_y_blur", dbg["y_blur"], manifest, entry)
        manifest["cases"][name] = entry
        o.close()
    with open(os.path.join(HERE, "manifest.json"), "w") as f:
        json.dump(manifest, f, indent=1, sort_keys=True)
    total = sum(os.path.getsize(os.path.join(HERE, x)) for x in os.listdir(HERE) if x.endswith(".bin"))
    print(f"wrote {len(manifest['cases'])} cases, {total / 1e6:.2f} MB")


if __name__ == "__main__":
    main()
