#!/usr/bin/env python3
"""Statistical profile of 10^4 concurrent per-call pipelines (one asyncio.gather):
a wall-clock interval timer (ITIMER_REAL: high-resolution, where the CPU-time timers
tick at the scheduler's rate) samples the running Python stack every ``AHV_SAMPLE_US``
µs of the CPU-bound run, so the split between the API's Python, its native calls
(attributed to the calling line) and asyncio carries no per-call profiler
overhead (cProfile roughly doubles the cost of short calls).

    DEV=cuda N=10000 python scripts/sample_gather.py
"""

from __future__ import annotations

import asyncio
import collections
import json
import os
import signal
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main() -> None:
    n = int(os.environ.get("N", "10000"))
    dev = os.environ.get("DEV", "cuda")
    period = int(os.environ.get("AHV_SAMPLE_US", "100"))
    from benchmarks.bench_api import reference_pipeline
    from hypervisor.config import tune_gc

    async def batch(k):
        return await asyncio.gather(*[reference_pipeline(dev) for _ in range(k)])

    tune_gc()
    asyncio.run(batch(500))
    lines: collections.Counter = collections.Counter()
    funcs: collections.Counter = collections.Counter()
    stacks: collections.Counter = collections.Counter()
    total = [0]

    def short(code) -> str:
        f = code.co_filename
        parts = f.split("/")
        return "/".join(parts[-2:])

    busy = [False]

    def on_sample(signum, frame):
        if busy[0]:  # a tick that lands inside the handler itself is not a sample
            return
        busy[0] = True
        try:
            record(frame)
        finally:
            busy[0] = False

    def record(frame):
        total[0] += 1
        if frame is None:
            return
        lines[f"{short(frame.f_code)}:{frame.f_lineno} {frame.f_code.co_name}"] += 1
        seen = set()
        f = frame
        chain = []
        while f is not None:
            key = f"{short(f.f_code)}:{f.f_code.co_name}"
            if key not in seen:
                funcs[key] += 1
                seen.add(key)
            if len(chain) < 4:
                chain.append(key)
            f = f.f_back
        stacks[" <- ".join(chain)] += 1

    signal.signal(signal.SIGALRM, on_sample)
    t_cpu = time.process_time()
    t0 = time.perf_counter()
    async def sampled():
        # the timer runs inside the loop only (a signal during loop setup breaks it)
        signal.setitimer(signal.ITIMER_REAL, period / 1e6, period / 1e6)
        try:
            return await batch(n)
        finally:
            signal.setitimer(signal.ITIMER_REAL, 0, 0)

    asyncio.run(sampled())
    dt = time.perf_counter() - t0
    cpu = time.process_time() - t_cpu
    us_per = dt / n * 1e6  # samples are of wall time (the run is host-CPU bound)
    out = {"device": dev, "pipelines": n, "pipelines_per_s": round(n / dt, 1),
           "cpu_us_per_pipeline": round(cpu / n * 1e6, 2),
           "wall_us_per_pipeline": round(us_per, 2),
           "samples": total[0]}
    print(json.dumps(out))

    def show(title, ctr, k):
        print(f"== {title} (µs of wall per pipeline, inclusive for functions)")
        for key, c in ctr.most_common(k):
            print(f"{c / max(total[0], 1) * us_per:8.2f}  {key}")

    show("lines (innermost Python frame)", lines, 45)
    show("functions", funcs, 45)
    show("stacks", stacks, 25)


if __name__ == "__main__":
    main()
