"""bench.py host logic on the CPU: the metric string, the frame-level roofline
arithmetic and the CPU-baseline child process (the oracle, bounded sample)."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def test_metric_matches_baseline_json_at_default_config():
    base = json.load(open(os.path.join(ROOT, "BASELINE.json")))["metric"]
    assert bench.metric_name(1920, 1080, 5) == base
    assert "3840×2160" in bench.metric_name(3840, 2160, 6)
    assert "8-orientation" in bench.metric_name(1920, 1080, 5, orientations=8)


def test_frame_roofline_is_sum_of_compulsory_bytes():
    W, H, N, C = 1920, 1080, 2048, 100
    cb = bench.compulsory_bytes(W, H, N, C)
    unfused = ["k_rows_fwd", "k_cols", "k_rows_inv", "k_compose"]
    fused = ["k_rows_fwd", "k_cols", "k_rows_inv_compose"]
    for ran, lo, hi in ((unfused, 70e6, 85e6), (fused, 55e6, 65e6)):
        r = bench.frame_roofline(W, H, N, 10000.0, C, ran=ran)
        per = sum(cb[k] for k in ran) / C
        assert r["bytes_per_frame"] == int(per)
        assert abs(r["frac"] - per * 1e4 / 8e12) < 1e-4
        # 1080p RGBA8: ~77 MB per frame through Yh, ~61 MB with K3+K4 fused
        # (DESIGN.md §5), far below SURVEY's 226 MB
        assert lo < per < hi
    # default: the unfused set
    assert bench.frame_roofline(W, H, N, 1e4, C)["bytes_per_frame"] == int(sum(cb[k] for k in unfused) / C)


def test_available_cpus_positive():
    assert 1 <= bench.available_cpus() <= (os.cpu_count() or 1)


def test_cpu_worker_runs_oracle(tmp_path):
    out = str(tmp_path / "w.json")
    subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--cpu-worker", "--cpu-out", out,
                    "--cpu-threads", "2", "--cpu-frames", "2", "--cpu-seconds", "30",
                    "--width", "64", "--height", "48", "--levels", "4", "--cpu-keep"],
                   check=True, timeout=120)
    rec = json.load(open(out))
    assert rec["frames"] == 2 and rec["threads"] == 2 and rec["seconds"] > 0
    import numpy as np
    outs = np.load(out + ".npy")
    assert outs.shape == (3, 48, 64, 4) and outs.dtype == np.uint8
