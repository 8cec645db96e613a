"""The reference's own test suite as an oracle.

``/root/reference/tests`` (326 tests: unit + integration, written for the
reference's pure-Python package) is run unmodified against this framework's
``hypervisor`` package — same import paths, same public API.  Nothing is copied
from the reference: pytest runs its test files in place (read-only, no cache or
bytecode written) with this repository first on ``PYTHONPATH`` and this repo's
minimal async plugin standing in for pytest-asyncio (not installed here).
Skipped when the reference checkout is not mounted (e.g. on the GPU box).
"""

from __future__ import annotations

import os
import re
import subprocess
import sys

import pytest

REF_TESTS = "/root/reference/tests"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.slow
@pytest.mark.skipif(not os.path.isdir(REF_TESTS), reason="reference checkout not mounted")
def test_reference_suite_passes_against_this_package():
    env = {k: v for k, v in os.environ.items() if k != "PYTHONPATH"}
    env.update(PYTHONPATH=ROOT, PYTHONDONTWRITEBYTECODE="1", AHV_SKIP_AUTOBUILD="1")
    cmd = [sys.executable, "-m", "pytest", REF_TESTS, "-q", "-p", "agent_hypervisor_amd.utils.pytest_async",
           "-p", "no:cacheprovider", "-c", os.devnull, "--rootdir", "/tmp"]
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=900, env=env, cwd="/tmp")
    tail = p.stdout[-3000:]
    assert p.returncode == 0, tail + p.stderr[-2000:]
    m = re.search(r"(\d+) passed", tail)
    assert m and int(m.group(1)) >= 326, tail
    assert "failed" not in tail and "error" not in tail.lower().split("passed")[-1], tail
