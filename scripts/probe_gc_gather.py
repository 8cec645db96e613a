#!/usr/bin/env python3
"""Cyclic-GC share of the 10^4-concurrent per-call gather (benchmarks/bench_api.py):
pipelines/s and the time spent in collections (gc.callbacks) per generation, for
the serving thresholds (tune_gc), the same after gc.freeze() of everything alive
after warm-up, and with the collector off (the bound).

    DEV=cuda N=10000 python scripts/probe_gc_gather.py
"""

from __future__ import annotations

import asyncio
import gc
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main() -> None:
    n = int(os.environ.get("N", "10000"))
    dev = os.environ.get("DEV", "cuda")
    from benchmarks.bench_api import reference_pipeline
    from hypervisor.config import tune_gc

    async def batch(k):
        return await asyncio.gather(*[reference_pipeline(dev) for _ in range(k)])

    tune_gc()
    asyncio.run(batch(500))
    acc = {"t": 0.0, "n": [0, 0, 0], "s": [0.0, 0.0, 0.0]}
    t0 = [0.0]

    def cb(phase, info):
        if phase == "start":
            t0[0] = time.perf_counter()
        else:
            dt = time.perf_counter() - t0[0]
            g = info["generation"]
            acc["n"][g] += 1
            acc["s"][g] += dt

    gc.callbacks.append(cb)
    for mode in ("tuned", "frozen", "off"):
        if mode == "frozen":
            gc.collect()
            gc.freeze()
        if mode == "off":
            gc.disable()
        for rep in range(2):
            acc["n"], acc["s"] = [0, 0, 0], [0.0, 0.0, 0.0]
            gc.collect() if mode != "off" else None
            acc["n"], acc["s"] = [0, 0, 0], [0.0, 0.0, 0.0]
            t = time.perf_counter()
            asyncio.run(batch(n))
            dt = time.perf_counter() - t
            print(json.dumps({"device": dev, "mode": mode, "rep": rep, "pipelines_per_s": round(n / dt, 1),
                              "us_per_pipeline": round(dt / n * 1e6, 2),
                              "gc_us_per_pipeline": round(sum(acc["s"]) / n * 1e6, 2),
                              "collections": acc["n"], "gc_ms_by_gen": [round(x * 1e3, 2) for x in acc["s"]],
                              "threshold": gc.get_threshold(), "frozen": gc.get_freeze_count()}), flush=True)
        if mode == "off":
            gc.enable()
    gc.callbacks.remove(cb)


if __name__ == "__main__":
    main()
