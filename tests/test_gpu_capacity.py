"""The capacity sweep's kernels at small sizes on the GPU (benchmarks/bench_capacity.py)."""

from __future__ import annotations

import os
import sys

import pytest

pytestmark = pytest.mark.gpu
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "benchmarks"))


def test_capacity_sweep_small(cuda_device):
    import bench_capacity as B

    r = B.liability(1 << 16, reps=2)
    assert r["edges"] == 4 << 16 and r["exposure_us"] > 0 and 0 < r["clip_pairs"] <= 16 * r["slash_k"]
    p = B.pipeline(1 << 16, reps=2)
    assert p["ok"] and p["sessions_per_s"] > 0
