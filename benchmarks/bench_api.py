#!/usr/bin/env python3
"""Concurrent public-API throughput (BASELINE config 2: "10k concurrent sessions").

N reference pipelines (``benchmarks/bench_hypervisor.py:217-239`` of the
reference: Hypervisor() → create → join → activate → 3 captures → saga
create/add/execute → terminate) run concurrently under one ``asyncio.gather``
through the public API.  With ``device="cuda"`` every call is a command to the
gfx950 store worker; awaited results suspend the calling pipeline (the other
pipelines keep issuing commands) and the hash engine compresses queued captures
of distinct sessions one per lane.  ``device="host"`` runs the same harness on
the pure host engines for comparison.

    python benchmarks/bench_api.py --device cuda --n 10000 --rounds 3
"""

from __future__ import annotations

import argparse
import asyncio
import gc
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


async def reference_pipeline(device: str) -> str:
    from hypervisor import Hypervisor, SessionConfig
    from hypervisor.audit.delta import VFSChange

    hv = Hypervisor(device=device)
    s = await hv.create_session(config=SessionConfig(enable_audit=True), creator_did="did:mesh:admin")
    sid = s.sso.session_id
    await hv.join_session(sid, "did:mesh:a", sigma_raw=0.8)
    await hv.activate_session(sid)
    for i in range(3):
        s.delta_engine.capture("did:mesh:a", [VFSChange(path=f"/f{i}", operation="add", content_hash=f"h{i}")])
    saga = s.saga.create_saga(sid)
    step = s.saga.add_step(saga.saga_id, "action", "did:mesh:a", "/api/action")
    await s.saga.execute_step(saga.saga_id, step.step_id, executor=lambda: asyncio.sleep(0))
    return await hv.terminate_session(sid)


def api_throughput(device: str, n: int = 10_000, rounds: int = 3, warm: int = 500) -> dict:
    """Pipelines/s of ``n`` concurrent reference pipelines (median of ``rounds``)."""

    async def batch(k):
        return await asyncio.gather(*[reference_pipeline(device) for _ in range(k)])

    from hypervisor.config import tune_gc

    old = tune_gc()  # the serving process's collector thresholds (AHV_GC_THRESHOLD), same for both paths
    asyncio.run(batch(warm))
    rates = []
    roots_ok = True
    for _ in range(rounds):
        gc.collect()
        t0 = time.perf_counter()
        roots = asyncio.run(batch(n))
        dt = time.perf_counter() - t0
        rates.append(n / dt)
        roots_ok = roots_ok and all(r is not None and len(r) == 64 for r in roots)
        # every pipeline computes the same chain shape but distinct ids → distinct roots
        roots_ok = roots_ok and len(set(roots)) == n
    gc.set_threshold(*old)
    return {"device": device, "concurrent_pipelines": n, "pipelines_per_s": round(statistics.median(rates), 1),
            "rounds": [round(r, 1) for r in rates], "roots_ok": roots_ok}


def batch_api_throughput(device: str, n: int = 100_000, rounds: int = 3, hetero: bool = False,
                         seed: int = 5) -> dict:
    """Sessions/s of :meth:`Hypervisor.run_pipelines` — the public batched API over
    the device store: every session is a complete pipeline written into store rows
    (create → join → activate → 3 audit deltas → saga step → terminate with its
    Merkle root committed) and an ordinary session of the hypervisor afterwards.
    ``hetero``: a randomized mix (1–5 joins with per-agent σ, 0–4 deltas of 0–3
    changes, 0–3 steps with retries/failures/compensation) instead of the template."""
    import random

    from agent_hypervisor_amd.models.store_pipeline import PipelineSpec
    from hypervisor import Hypervisor

    if hetero:
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        from test_store_pipeline import random_spec

        rng = random.Random(seed)
        specs = [random_spec(rng) for _ in range(n)]
    else:
        specs = PipelineSpec()

    marks: dict = {}

    async def one():
        t = time.perf_counter()
        hv = Hypervisor(device=device)
        marks["init"] = time.perf_counter() - t
        r = await hv.run_pipelines(specs, None if hetero else n)
        marks["teardown0"] = time.perf_counter()
        return r

    asyncio.run(one())  # warm-up (allocations, kernel load)
    rates, dev, phases = [], [], []
    ok = True
    for _ in range(rounds):
        gc.collect()
        t0 = time.perf_counter()
        run = asyncio.run(one())
        dt = time.perf_counter() - t0
        rates.append(n / dt)
        dev.append(run.device_seconds)
        phases.append({"hv_init": marks["init"], "prepare": run.prepare_seconds, "device": run.device_seconds,
                       "finish": run.finish_seconds, "teardown": time.perf_counter() - marks["teardown0"]})
        ok = ok and (hetero or (run.ok == n and len(run.roots) == n))
    return {"device": device, "sessions": n, "hetero": hetero, "sessions_per_s": round(statistics.median(rates), 1),
            "rounds": [round(r, 1) for r in rates], "device_ms": [round(1000 * x, 2) for x in dev],
            "phases_ms": {k: round(1000 * statistics.median(p[k] for p in phases), 2) for k in phases[0]}, "ok": ok}


def main() -> None:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--device", default="cuda")
    ap.add_argument("--n", type=int, default=10_000)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--host", action="store_true", help="also run the host engines for comparison")
    ap.add_argument("--batch", type=int, default=0, help="also time run_pipelines over this many sessions")
    args = ap.parse_args()
    out = {}
    if args.n:
        out["device"] = api_throughput(args.device, args.n, args.rounds)
        if args.host:
            out["host"] = api_throughput("host", args.n, args.rounds)
    if args.batch:
        out["batch"] = batch_api_throughput(args.device, args.batch, args.rounds)
        out["batch_hetero"] = batch_api_throughput(args.device, args.batch, args.rounds, hetero=True)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
