"""Thousands of concurrent reference pipelines through one device store.

Regression: the saga step's posted EXECUTING transition is awaited only after the
executor ran, by which time thousands of other sessions' commands may have been
posted and its result slot recycled ("store result slot recycled").  Posted
results that are read later are kept (``GovernanceStore.post(..., keep=True)``).
"""

from __future__ import annotations

import asyncio
import os
import sys

import pytest

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "benchmarks"))

from bench_api import reference_pipeline  # noqa: E402


def _gather(device: str, n: int) -> list:
    async def go():
        return await asyncio.gather(*[reference_pipeline(device) for _ in range(n)])

    return asyncio.run(go())


def test_concurrent_pipelines_cpu_twin():
    roots = _gather("cpu", 3000)
    assert len(roots) == 3000 and len(set(roots)) == 3000 and all(len(r) == 64 for r in roots)


@pytest.mark.gpu
def test_concurrent_pipelines_gfx950():
    roots = _gather("cuda", 5000)
    assert len(roots) == 5000 and len(set(roots)) == 5000 and all(len(r) == 64 for r in roots)
