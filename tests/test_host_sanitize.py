"""Host-side ASan + UBSan run of the kernel library's launch planners.

Builds tools/host_sanitize.cpp against the csrc/ objects with ``-Xarch_host -fsanitize=...``
(scripts/host_sanitize.sh) and runs the geometry sweep on the CPU.  No GPU is used."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("hipcc") is None, reason="hipcc not available")
def test_planners_clean_under_asan_ubsan(tmp_path):
    env = dict(os.environ, OUT=str(tmp_path / "san"))
    r = subprocess.run(["bash", os.path.join(ROOT, "scripts", "host_sanitize.sh")], cwd=ROOT,
                       env=env, capture_output=True, text=True, timeout=900)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert "planner checks passed" in r.stdout
