"""The CPU-side C code under AddressSanitizer + UndefinedBehaviorSanitizer
(SURVEY.md §5): the oracle (oracle/mm_ref.c) and the C driver's Y4M module
(host/y4m.c) built together with tests/sanitize/san_check.c, any finding fatal
(-fno-sanitize-recover=all; LeakSanitizer on).  Host code only: GPU sanitizers
are not available on this pool."""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_oracle_and_y4m_clean_under_asan_ubsan(tmp_path):
    exe = str(tmp_path / "san_check")
    subprocess.run(["gcc", "-std=gnu11", "-O1", "-g", "-fopenmp", "-fsanitize=address,undefined",
                    "-fno-sanitize-recover=all", "-fno-omit-frame-pointer",
                    "-I", os.path.join(ROOT, "oracle"),
                    "-I", os.path.join(ROOT, "phase-based-motion-manipulation_amd", "host"),
                    "-o", exe, os.path.join(ROOT, "tests", "sanitize", "san_check.c"),
                    os.path.join(ROOT, "oracle", "mm_ref.c"),
                    os.path.join(ROOT, "phase-based-motion-manipulation_amd", "host", "y4m.c"), "-lm"],
                   check=True, timeout=300)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0",
               UBSAN_OPTIONS="print_stacktrace=1", OMP_NUM_THREADS="2")
    r = subprocess.run([exe], capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, r.stdout + r.stderr[-4000:]
    assert "san_check: ok" in r.stdout
    assert "runtime error" not in r.stderr and "AddressSanitizer" not in r.stderr
