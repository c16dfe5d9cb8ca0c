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


def test_cpu_worker_boundary_pairs_equal_sequential(tmp_path):
    """The boundary frames the bench's parity check adds (oracle reset, fed
    frames t-1 and t) equal the sequential oracle's frame t: output t depends
    only on inputs t-1 and t (.cs:142)."""
    import numpy as np
    out = str(tmp_path / "w.json")
    subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--cpu-worker", "--cpu-out", out,
                    "--cpu-threads", "2", "--cpu-frames", "5", "--cpu-seconds", "60",
                    "--width", "64", "--height", "48", "--levels", "5", "--cpu-keep",
                    "--cpu-pairs", "2,5"], check=True, timeout=120)
    seq = np.load(out + ".npy")
    pairs = np.load(out + ".pairs.npy")
    assert np.array_equal(pairs[0], seq[2]) and np.array_equal(pairs[1], seq[5])


def test_boundary_frames_cover_k2_launch_shapes():
    """300 frames in batches of 150 at 1080p: each batch's prime, the packed
    block's hand-off to k_cols_tail (40 %: frame 90 of a batch), the second-half
    tails (10 %: frame 135) and the batch ends; frames 1..30 are sequential."""
    b = bench.boundary_frames(300, 150, 1920, 1080)
    for t in (89, 90, 134, 135, 149, 150, 151, 239, 240, 284, 285, 299):
        assert t in b
    assert all(31 <= t < 300 for t in b)
    # 2160p: 30 % tails
    assert 105 in bench.boundary_frames(300, 150, 3840, 2160)
