"""The host-only C++ under AddressSanitizer + UndefinedBehaviorSanitizer and under
ThreadSanitizer: `make -C proxmox-backup_amd/csrc sanitize` builds
tests/cpp/host_sanitize.cpp with the SHA lanes (pbs_sha_host.cpp), the pipeline's host
share (csrc/host_share.h: routing, worker pool, zero-chunk memo, per-chunk flags) and the
.didx writer, and runs both builds; any sanitizer report fails the run (halt_on_error).
No device is involved."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("g++") is None, reason="no g++")
def test_host_cpp_under_sanitizers(tmp_path):
    r = subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "proxmox-backup_amd", "csrc"), "sanitize"],
                       capture_output=True, text=True, timeout=600)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-4000:]
    assert out.count("host_sanitize ok (0 failures)") == 2, out[-4000:]
    assert "ERROR: AddressSanitizer" not in out and "WARNING: ThreadSanitizer" not in out
