"""Host-side index math under AddressSanitizer + UndefinedBehaviorSanitizer (CPU only): FA2 block
orders are bijections, the LDS swizzles stay in-row and bank-conflict free, Tensile name parsing
(csrc/tests/host_checks.cpp via scripts/sanitize_host.sh)."""

import os
import shutil
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("hipcc") is None and not os.path.exists("/opt/rocm/bin/hipcc"), reason="needs hipcc")
def test_host_checks_under_asan_ubsan(tmp_path):
    env = dict(os.environ, TMPDIR=str(tmp_path), PATH=os.environ.get("PATH", "") + ":/opt/rocm/bin")
    r = subprocess.run(["bash", "scripts/sanitize_host.sh"], cwd=REPO, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert "host checks passed" in r.stdout
