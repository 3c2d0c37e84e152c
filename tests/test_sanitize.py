"""Host code under AddressSanitizer + UndefinedBehaviorSanitizer (`make sanitize`): the CPU oracle
and the facade's host-only paths (POSCAR parser, Structure, PCA) on the committed fixtures. CPU only."""
import shutil
import subprocess

import pytest
from conftest import ROOT


@pytest.mark.skipif(shutil.which("g++") is None, reason="no host compiler")
def test_make_sanitize_clean():
    r = subprocess.run(["make", "-s", "sanitize"], cwd=ROOT, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert "san_check ok" in r.stdout
    assert "runtime error" not in r.stderr and "AddressSanitizer" not in r.stderr
