"""Host runtime under AddressSanitizer+UBSan and ThreadSanitizer.

Builds csrc/host (no HIP) + csrc/tests/host_selftest.cpp with g++ -fsanitize=... and runs the
self-test, which drives the threaded CPU miner (brute-force checked), the threaded rule engine,
the matcher, the multi-threaded generator and the CSV ingest."""
import pathlib
import shutil
import subprocess

import pytest

ROOT = pathlib.Path(__file__).resolve().parents[1]


@pytest.mark.skipif(shutil.which("g++") is None, reason="g++ not available")
@pytest.mark.parametrize("mode", ["asan", "tsan"])
def test_host_selftest_sanitized(mode):
    r = subprocess.run(["bash", str(ROOT / "scripts" / "sanitize_host.sh"), mode],
                       capture_output=True, text=True, timeout=900)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert "host selftest OK" in r.stdout
