#!/usr/bin/env python3
"""Where the time of N concurrent per-call pipelines (one asyncio.gather) goes.

Prints one JSON object per run: pipelines/s, host CPU µs per pipeline, the
store worker's busy µs per pipeline (command wave, hash engine), commands per
pipeline, then the top host functions by own time (cProfile over one round)."""

from __future__ import annotations

import asyncio
import cProfile
import gc
import io
import json
import os
import pstats
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
    st = None
    if dev != "host":
        from hypervisor import _device

        st = _device._shared_store(dev)
    for rnd in range(2):
        gc.collect()
        i0 = st.info() if st else {}
        c0, w0 = time.process_time(), time.perf_counter()
        asyncio.run(batch(n))
        wall, cpu = time.perf_counter() - w0, time.process_time() - c0
        i1 = st.info() if st else {}
        d = {k: i1[k] - i0[k] for k in i1 if isinstance(i1.get(k), (int, float)) and isinstance(i0.get(k), (int,
                                                                                                            float))}
        print(json.dumps({
            "device": dev, "round": rnd, "pipelines": n, "pipelines_per_s": round(n / wall, 1),
            "host_cpu_us_per_pipeline": round(cpu / n * 1e6, 2),
            "worker_busy_us_per_pipeline": round(d.get("worker_busy_us", 0) / n, 2),
            "engine_busy_us_per_pipeline": round(d.get("engine_busy_us", 0) / n, 2),
            "commands_per_pipeline": round(d.get("posted", 0) / n, 3),
            "engine_jobs_per_pipeline": round(d.get("engine_jobs", 0) / n, 3),
            "ring_wait_us_per_pipeline": round(d.get("ring_wait_us", 0) / n, 2),
        }), flush=True)
    pr = cProfile.Profile()
    pr.enable()
    asyncio.run(batch(n // 4))
    pr.disable()
    s = io.StringIO()
    pstats.Stats(pr, stream=s).sort_stats(os.environ.get("SORT", "tottime")).print_stats(int(os.environ.get("TOP",
                                                                                                            "30")))
    print("\n".join(ln for ln in s.getvalue().splitlines() if ln.strip()))


if __name__ == "__main__":
    main()
