"""The CPU restatement under AddressSanitizer + UndefinedBehaviorSanitizer:
`make -C oracle asan-run` builds refcpu.cpp with -fsanitize=address,undefined (host code
only) together with oracle/asan_check.cpp, which drives every entry point — all run kinds
and estimators with the per-iteration trace, trimmed and untrimmed, kNN at k = 30 / 90 /
150, TOLDI frames, normals, GICP covariances, 3-D and 12-D NN, the estimators and the
trimmed rejector — on the reference fixture and checks the analytic ground truth.  Any
sanitizer finding aborts the run."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++ with libasan")
def test_oracle_under_asan_and_ubsan():
    r = subprocess.run(["make", "-C", os.path.join(ROOT, "oracle"), "asan-run"], capture_output=True, text=True,
                       timeout=600)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-4000:]
    assert "ok: 0 failures" in out
    assert "ERROR: AddressSanitizer" not in out and "runtime error" not in out
