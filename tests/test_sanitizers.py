"""§5.2: the native host code (every kernel's host twin, the pipeline emitter,
hashing) under AddressSanitizer + UndefinedBehaviorSanitizer.

Compiling the sanitizer build takes ~2 minutes, so it runs when
``AHV_RUN_SANITIZERS=1`` (CI sets it); otherwise the test is skipped."""

from __future__ import annotations

import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.slow
@pytest.mark.skipif(os.environ.get("AHV_RUN_SANITIZERS") != "1", reason="set AHV_RUN_SANITIZERS=1")
def test_host_selftest_under_asan_ubsan():
    p = subprocess.run(["bash", os.path.join(ROOT, "scripts", "sanitize_host.sh")], capture_output=True, text=True,
                       timeout=1800, cwd=ROOT)
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-4000:]
    assert "all checks passed" in p.stdout
