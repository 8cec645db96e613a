#!/usr/bin/env python3
"""Where the per-call device path spends its CPU: cProfile of N concurrent reference
pipelines (benchmarks/bench_api.py) on one device, printed top-K by self time,
plus the unprofiled rate for the same N.

    python scripts/api_percall_prof.py --device cuda --n 10000
"""

from __future__ import annotations

import argparse
import asyncio
import cProfile
import io
import json
import os
import pstats
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from benchmarks.bench_api import reference_pipeline  # noqa: E402
from hypervisor.config import tune_gc  # noqa: E402


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--device", default="cuda")
    ap.add_argument("--n", type=int, default=10_000)
    ap.add_argument("--top", type=int, default=30)
    a = ap.parse_args()
    tune_gc()

    async def batch(k):
        return await asyncio.gather(*[reference_pipeline(a.device) for _ in range(k)])

    asyncio.run(batch(500))
    t = time.perf_counter()
    asyncio.run(batch(a.n))
    rate = a.n / (time.perf_counter() - t)
    print(json.dumps({"device": a.device, "n": a.n, "pipelines_per_s": round(rate, 1)}), flush=True)
    pr = cProfile.Profile()
    pr.enable()
    asyncio.run(batch(a.n))
    pr.disable()
    s = io.StringIO()
    pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(a.top)
    print(s.getvalue(), flush=True)


if __name__ == "__main__":
    main()
