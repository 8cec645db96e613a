#!/usr/bin/env python3
"""Batched public API: many sessions' governance pipelines in one call.

``Hypervisor.run_pipelines`` writes every session's pipeline — create, joins
(ring gate + admission), activate, audit deltas (canonical records, SHA-256
chain), saga steps (retries, failure, compensation), terminate (Merkle root
committed) — straight into the device store's rows with three gfx950 kernels
(``csrc/hip/store_pipeline.hip``).  The sessions are ordinary sessions of the
hypervisor afterwards: ``get_session`` builds their views on first use, and
``verify_audit``, snapshots, the REST routes and the dashboard read them where
they live.

    python examples/batch_pipelines.py            # GPU if present, else the CPU twin
"""

from __future__ import annotations

import asyncio
import os
import random
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from agent_hypervisor_amd.models.store_pipeline import PipelineSpec  # noqa: E402
from hypervisor import Hypervisor  # noqa: E402


def spec(rng: random.Random, i: int) -> PipelineSpec:
    agents = [f"did:mesh:agent{(i + k) % 50}" for k in range(rng.randint(1, 3))]
    return PipelineSpec(
        joins=[(a, rng.choice([0.3, 0.65, 0.8, 0.97])) for a in agents],
        deltas=[(rng.choice(agents), [(f"/doc/{i}/{k}", "add", f"sha256:{rng.getrandbits(64):016x}")])
                for k in range(rng.randint(0, 3))],
        steps=[(f"action{k}", agents[0], "/api/run", "/api/undo" if rng.random() < 0.9 else None,
                rng.choice([0, 1]), rng.choice([0, 0, 1, 5])) for k in range(rng.randint(0, 2))],
    )


async def main() -> None:
    device = "cuda" if torch.cuda.is_available() else "cpu"
    hv = Hypervisor(device=device)
    t = time.perf_counter()
    run = await hv.run_pipelines(PipelineSpec(), 20_000)  # the reference pipeline, 2·10⁴ sessions
    print(f"template: {run.ok} sessions ok in {1e3 * (time.perf_counter() - t):.1f} ms "
          f"(device {1e3 * run.device_seconds:.2f} ms), {len(run.roots)} Merkle roots committed")
    rng = random.Random(7)
    specs = [spec(rng, i) for i in range(5_000)]
    run = await hv.run_pipelines(specs)
    names = {}
    for i in range(len(specs)):
        names[run.status_name(i)] = names.get(run.status_name(i), 0) + 1
    print("heterogeneous:", dict(sorted(names.items())))
    sid = run.session_ids[0]
    m = hv.get_session(sid)  # views built now, over the same rows
    print(sid, m.sso.state.value, [p.agent_did for p in m.sso.participants], len(m.delta_engine.deltas), "deltas")
    rep = hv.verify_audit()  # K10/K09 over the resident rows
    print(f"verify_audit: ok={rep.ok} over {rep.sessions} sessions, {rep.deltas} deltas, {rep.roots_checked} roots")


if __name__ == "__main__":
    asyncio.run(main())
