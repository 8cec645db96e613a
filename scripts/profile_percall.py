#!/usr/bin/env python3
"""Where the time of one per-call device pipeline goes (Hypervisor(device="cuda")).

Prints one JSON object: p50/mean of the reference-harness pipeline, host CPU
time per pipeline (process time), the wall time spent waiting on the
terminate command (the Merkle root needs every capture hashed), the worker's
busy time per pipeline (store telemetry), and the top host functions by own
time (cProfile over a shorter run)."""

from __future__ import annotations

import asyncio
import cProfile
import io
import json
import os
import pstats
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main() -> None:
    iters = int(os.environ.get("ITERS", "2000"))
    dev = os.environ.get("DEV", "cuda")
    from hypervisor import Hypervisor, SessionConfig
    from hypervisor import core as hcore
    from hypervisor.audit.delta import VFSChange

    waits = []
    orig = hcore.Hypervisor._terminate_device

    async def timed_terminate(self, sid, managed):
        t0 = time.perf_counter_ns()
        try:
            return await orig(self, sid, managed)
        finally:
            waits.append(time.perf_counter_ns() - t0)

    hcore.Hypervisor._terminate_device = timed_terminate

    async def one():
        hv = Hypervisor(device=dev)
        s = await hv.create_session(config=SessionConfig(enable_audit=True), creator_did="did:mesh:admin")
        sid = s.sso.session_id
        await hv.join_session(sid, "did:mesh:a", sigma_raw=0.8)
        await hv.activate_session(sid)
        for i in range(3):
            s.delta_engine.capture("did:mesh:a", [VFSChange(path=f"/f{i}", operation="add", content_hash=f"h{i}")])
        saga = s.saga.create_saga(sid)
        step = s.saga.add_step(saga.saga_id, "action", "did:mesh:a", "/api/action")
        await s.saga.execute_step(saga.saga_id, step.step_id, executor=lambda: asyncio.sleep(0))
        await hv.terminate_session(sid)

    async def run(n):
        lat = []
        for _ in range(n):
            t0 = time.perf_counter_ns()
            await one()
            lat.append(time.perf_counter_ns() - t0)
        return lat

    asyncio.run(run(200))
    waits.clear()
    from hypervisor import _device

    st = _device._shared_store(dev)
    tel0 = list(st._c.tail)[:5] if hasattr(st._c, "tail") else None
    import gc

    gc_t = {"n": [0, 0, 0], "ns": [0, 0, 0], "t0": 0}

    def on_gc(phase, info):  # time spent in the cyclic collector, per generation
        if phase == "start":
            gc_t["t0"] = time.perf_counter_ns()
        else:
            g = info.get("generation", 0)
            gc_t["n"][g] += 1
            gc_t["ns"][g] += time.perf_counter_ns() - gc_t["t0"]

    gc.callbacks.append(on_gc)
    info0 = st.info()
    c0 = time.process_time()
    w0 = time.perf_counter()
    lat = asyncio.run(run(iters))
    wall = time.perf_counter() - w0
    cpu = time.process_time() - c0
    info1 = st.info()
    gc.callbacks.remove(on_gc)
    srt = sorted(lat)
    pr = cProfile.Profile()
    pr.enable()
    asyncio.run(run(300))
    pr.disable()
    s = io.StringIO()
    pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(25)
    top = [ln for ln in s.getvalue().splitlines() if ln.strip()][:40]
    out = {
        "device": dev, "iters": iters, "p50_us": statistics.median(lat) / 1e3, "mean_us": statistics.mean(lat) / 1e3,
        "host_cpu_us_per_pipeline": cpu / iters * 1e6, "wall_us_per_pipeline": wall / iters * 1e6,
        "terminate_wait_p50_us": statistics.median(waits[-iters:]) / 1e3 if waits else None,
        "p90_us": srt[int(0.9 * len(srt))] / 1e3, "p99_us": srt[int(0.99 * len(srt))] / 1e3, "max_us": srt[-1] / 1e3,
        "gc_collections": gc_t["n"], "gc_us_per_pipeline": sum(gc_t["ns"]) / iters / 1e3,
        "commands_per_pipeline": (info1.get("posted", 0) - info0.get("posted", 0)) / iters,
        "store_info_delta": {k: info1[k] - info0[k] for k in info1 if isinstance(info1.get(k), (int, float))
                             and isinstance(info0.get(k), (int, float))},
        "telemetry_before": tel0,
    }
    print(json.dumps(out))
    print("\n".join(top))


if __name__ == "__main__":
    main()
