#!/usr/bin/env python3
"""Scalar-API microbenchmarks with the reference harness's methodology.

The same nine operations and iteration counts as the reference's
benchmarks/bench_hypervisor.py (ring computation, vouching σ_eff, delta
capture, Merkle roots of 10/100 deltas, chain verify of 50, session lifecycle,
3-step saga, full governance pipeline) run against *this* package's public
API: warm-up of ``min(100, iters // 10)`` iterations, per-iteration
``perf_counter_ns``, executors stubbed with ``asyncio.sleep(0)``, throughput
``1e9 / mean``.  Results go to ``benchmarks/results/`` as JSON and markdown,
side by side with the reference's published numbers.

The batched device configurations (BASELINE configs 2–5) live in
``benchmarks/bench_configs.py``; the headline driver contract is ``bench.py``.
"""

from __future__ import annotations

import argparse
import asyncio
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from hypervisor import Hypervisor, SessionConfig  # noqa: E402
from hypervisor.audit.delta import DeltaEngine, VFSChange  # noqa: E402
from hypervisor.liability.vouching import VouchingEngine  # noqa: E402
from hypervisor.rings.enforcer import RingEnforcer  # noqa: E402
from hypervisor.saga.orchestrator import SagaOrchestrator  # noqa: E402

# Reference published p50 (µs) — BASELINE.md, benchmarks.json of the reference.
REFERENCE_P50_US = {
    "ring_computation": 0.2,
    "vouching_sigma_eff": 666.2,
    "delta_capture": 27.3,
    "merkle_root_10_deltas": 352.85,
    "merkle_root_100_deltas": 3381.45,
    "chain_verify_50_deltas": 2011.05,
    "session_lifecycle": 54.0,
    "saga_3_steps": 151.25,
    "full_governance_pipeline": 267.5,
}


def _summary(name: str, ns: list[int]) -> dict:
    s = sorted(ns)
    n = len(s)
    mean = statistics.mean(s)
    pick = lambda q: s[min(n - 1, int(q * n))] / 1000.0  # noqa: E731
    return {
        "name": name,
        "iterations": n,
        "mean_us": mean / 1000.0,
        "median_us": statistics.median(s) / 1000.0,
        "p95_us": pick(0.95),
        "p99_us": pick(0.99),
        "min_us": s[0] / 1000.0,
        "max_us": s[-1] / 1000.0,
        "ops_per_sec": int(1e9 / mean) if mean else 0,
        "reference_p50_us": REFERENCE_P50_US.get(name),
    }


def run_sync(name, fn, iters):
    for _ in range(min(100, iters // 10)):
        fn()
    out = []
    for _ in range(iters):
        t0 = time.perf_counter_ns()
        fn()
        out.append(time.perf_counter_ns() - t0)
    return _summary(name, out)


def run_async(name, fn, iters):
    async def go():
        for _ in range(min(100, iters // 10)):
            await fn()
        out = []
        for _ in range(iters):
            t0 = time.perf_counter_ns()
            await fn()
            out.append(time.perf_counter_ns() - t0)
        return out

    return _summary(name, asyncio.run(go()))


def build_suite(scale: float = 1.0):
    it = lambda n: max(10, int(n * scale))  # noqa: E731
    enforcer = RingEnforcer()
    ve = VouchingEngine()
    counter = [0]

    def ring():
        enforcer.compute_ring(0.85)

    def sigma_eff():
        counter[0] += 1
        k = counter[0]
        sid = f"bench-{k}"
        ve.vouch(f"did:v:{k}", f"did:e:{k}", sid, 0.9, bond_pct=0.2)
        ve.compute_sigma_eff(f"did:e:{k}", sid, 0.4, risk_weight=0.5)

    def capture():
        DeltaEngine("bench-session").capture("did:mesh:a", [VFSChange(path="/data/file.txt", operation="add",
                                                                      content_hash="abc123")])

    def merkle(n):
        def f():
            de = DeltaEngine("bench-merkle")
            for i in range(n):
                de.capture("did:mesh:a", [VFSChange(path=f"/f{i}", operation="add", content_hash=f"h{i}")])
            de.compute_merkle_root()
        return f

    def verify():
        de = DeltaEngine("bench-verify")
        for i in range(50):
            de.capture("did:mesh:a", [VFSChange(path=f"/f{i}", operation="add", content_hash=f"h{i}")])
        de.verify_chain()

    async def lifecycle():
        hv = Hypervisor()
        s = await hv.create_session(config=SessionConfig(), creator_did="did:mesh:admin")
        await hv.join_session(s.sso.session_id, "did:mesh:a", sigma_raw=0.8)
        await hv.activate_session(s.sso.session_id)
        await hv.terminate_session(s.sso.session_id)

    async def saga3():
        orch = SagaOrchestrator()
        saga = orch.create_saga("bench-session")
        steps = [orch.add_step(saga.saga_id, f"action{i}", f"did:mesh:{i}", f"/api/{i}", undo_api=f"/api/undo/{i}")
                 for i in range(3)]
        for st in steps:
            await orch.execute_step(saga.saga_id, st.step_id, executor=lambda: asyncio.sleep(0))

    async def pipeline():
        hv = Hypervisor()
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

    return [
        ("ring_computation", ring, it(50000), False),
        ("vouching_sigma_eff", sigma_eff, it(10000), False),
        ("delta_capture", capture, it(50000), False),
        ("merkle_root_10_deltas", merkle(10), it(10000), False),
        ("merkle_root_100_deltas", merkle(100), it(1000), False),
        ("chain_verify_50_deltas", verify, it(2000), False),
        ("session_lifecycle", lifecycle, it(5000), True),
        ("saga_3_steps", saga3, it(5000), True),
        ("full_governance_pipeline", pipeline, it(2000), True),
    ]


def main() -> None:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--scale", type=float, default=1.0, help="multiply iteration counts")
    ap.add_argument("--out", default=os.path.join(os.path.dirname(os.path.abspath(__file__)), "results"))
    ap.add_argument("--only", default="", help="comma-separated benchmark names")
    args = ap.parse_args()
    only = {x for x in args.only.split(",") if x}
    results = []
    for name, fn, iters, is_async in build_suite(args.scale):
        if only and name not in only:
            continue
        r = (run_async if is_async else run_sync)(name, fn, iters)
        ref = r["reference_p50_us"]
        speed = f"{ref / r['median_us']:.1f}x" if ref and r["median_us"] else "-"
        print(f"{name:28s} p50 {r['median_us']:10.2f} µs  mean {r['mean_us']:10.2f} µs  "
              f"{r['ops_per_sec']:>10,} ops/s  vs ref p50 {speed}", flush=True)
        results.append(r)
    os.makedirs(args.out, exist_ok=True)
    with open(os.path.join(args.out, "benchmarks.json"), "w") as f:
        json.dump({"benchmarks": results}, f, indent=2)
    with open(os.path.join(args.out, "BENCHMARKS.md"), "w", encoding="utf-8") as f:
        f.write("# Scalar-API microbenchmarks (reference harness methodology)\n\n")
        f.write("| Operation | Mean µs | P50 µs | P95 µs | P99 µs | ops/s | Reference P50 µs | Speed-up (P50) |\n")
        f.write("|---|---|---|---|---|---|---|---|\n")
        for r in results:
            ref = r["reference_p50_us"]
            f.write(f"| {r['name']} | {r['mean_us']:.2f} | {r['median_us']:.2f} | {r['p95_us']:.2f} | "
                    f"{r['p99_us']:.2f} | {r['ops_per_sec']:,} | {ref} | "
                    f"{ref / r['median_us']:.1f}x |\n")
    print(f"results written to {args.out}/")


if __name__ == "__main__":
    main()
