"""Shared pytest configuration.

* ``gpu`` marker: tests that need a real MI355X (run with ``-m gpu``).
* ``async def`` tests run through :mod:`agent_hypervisor_amd.utils.pytest_async`
  (pytest-asyncio is not available in this image).
* The native extension is (re)built in-tree before collection if stale.
"""

from __future__ import annotations

import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

pytest_plugins = ["agent_hypervisor_amd.utils.pytest_async"]


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: requires an AMD Instinct GPU (HIP device)")
    config.addinivalue_line("markers", "slow: long-running test")
    from agent_hypervisor_amd.utils import build

    if build.needs_build():
        build.build()


@pytest.fixture(autouse=True)
def _reset_clock_and_parity():
    from hypervisor import _clock, config

    yield
    _clock.set_clock(None)
    config.set_parity_mode(False)


def gpu_available() -> bool:
    try:
        import torch

        return torch.cuda.is_available()
    except Exception:
        return False


@pytest.fixture
def cuda_device():
    if not gpu_available():
        pytest.fail("GPU test selected but no HIP device is visible")
    import torch

    return torch.device("cuda", 0)
