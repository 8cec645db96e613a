#!/usr/bin/env python3
"""Live dashboard example (reference ``examples/dashboard/app.py``).

Starts the REST API with its ``/dashboard`` page (``hypervisor/api/dashboard.py``)
around a hypervisor that a background task keeps busy with a small, varied
workload — sessions joining at different σ (so every ring shows up), vouches and
a slash cascade, sagas that commit, fail and compensate, audit captures and
terminations — so every tab renders live state rather than synthetic data.

    python examples/dashboard/app.py --port 8000      # then open http://127.0.0.1:8000/dashboard
    python examples/dashboard/app.py --device cuda    # state authoritative on the GPU store
    python examples/dashboard/app.py --once           # run one workload round, print the summary, exit
"""

from __future__ import annotations

import argparse
import asyncio
import json
import os
import random
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

from hypervisor import Hypervisor, SessionConfig  # noqa: E402
from hypervisor.api.dashboard import summary  # noqa: E402
from hypervisor.api.server import ApiState, create_app  # noqa: E402
from hypervisor.audit.delta import VFSChange  # noqa: E402
from hypervisor.observability.event_bus import HypervisorEventBus  # noqa: E402


async def workload_round(hv: Hypervisor, rnd: random.Random, k: int) -> None:
    """One round: a session with 3–5 agents, vouches, captures, a saga, maybe a slash."""
    m = await hv.create_session(SessionConfig(min_sigma_eff=0.3), creator_did="did:mesh:admin")
    sid = m.sso.session_id
    agents = [f"did:mesh:agent-{k}-{j}" for j in range(rnd.randint(3, 5))]
    sigmas = {}
    for a in agents:
        sigmas[a] = round(rnd.uniform(0.35, 0.99), 3)
        await hv.join_session(sid, a, sigma_raw=sigmas[a])
    await hv.activate_session(sid)
    hi = max(agents, key=sigmas.get)
    for a in agents:
        if a != hi and sigmas[hi] >= 0.5:
            try:
                hv.vouching.vouch(hi, a, sid, sigmas[hi], bond_pct=0.15)
            except Exception:  # noqa: BLE001 - exposure limits are part of the demo
                pass
    for i in range(rnd.randint(1, 4)):
        m.sso.vfs.write(f"/work/{i}.txt", f"round {k} artefact {i}", agents[0])
        m.delta_engine.capture(agents[0], [VFSChange(path=f"/work/{i}.txt", operation="add", content_hash=f"c{k}.{i}")])
    saga = m.saga.create_saga(sid)
    steps = [m.saga.add_step(saga.saga_id, f"step{j}", agents[j % len(agents)], f"/api/s{j}",
                             undo_api=f"/api/u{j}" if j % 3 else None) for j in range(3)]
    fail_at = rnd.choice([None, None, 2])
    for j, st in enumerate(steps):
        async def run(j=j):
            if j == fail_at:
                raise RuntimeError("downstream API refused")
            return {"ok": j}
        try:
            await m.saga.execute_step(saga.saga_id, st.step_id, executor=run)
        except Exception:  # noqa: BLE001 - the failure drives compensation below
            await m.saga.compensate(saga.saga_id, lambda step: asyncio.sleep(0))
            break
    if k % 4 == 3:  # behavioural drift → slash cascade through the vouches
        victim = next((a for a in agents if a != hi), None)
        if victim:
            hv.slashing.slash(victim, sid, sigmas[victim], 0.95, "demo drift", dict(sigmas))
    if k % 2 == 0:
        await hv.terminate_session(sid)


async def keep_busy(hv: Hypervisor, period: float) -> None:
    rnd = random.Random(7)
    k = 0
    while True:
        await workload_round(hv, rnd, k)
        k += 1
        await asyncio.sleep(period)


def main() -> None:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--host", default="127.0.0.1")
    ap.add_argument("--port", type=int, default=8000)
    ap.add_argument("--device", default="host", help="host | cpu | cuda (state store)")
    ap.add_argument("--period", type=float, default=2.0, help="seconds between workload rounds")
    ap.add_argument("--once", action="store_true", help="one round of 8 sessions, print the summary, exit")
    args = ap.parse_args()
    bus = HypervisorEventBus()
    hv = Hypervisor(device=args.device, event_bus=bus)
    if args.once:
        async def go():
            rnd = random.Random(7)
            for k in range(8):
                await workload_round(hv, rnd, k)
        asyncio.run(go())
        print(json.dumps(summary(ApiState(bus=bus, hv=hv)), default=str)[:4000])
        return
    import uvicorn

    from contextlib import asynccontextmanager

    app = create_app(hv, bus)
    inner = app.router.lifespan_context

    @asynccontextmanager
    async def lifespan(application):  # the workload lives on the server's event loop
        async with inner(application):
            task = asyncio.get_running_loop().create_task(keep_busy(hv, args.period))
            try:
                yield
            finally:
                task.cancel()

    app.router.lifespan_context = lifespan
    uvicorn.run(app, host=args.host, port=args.port, log_level="warning")


if __name__ == "__main__":
    main()
