"""GPU probe of the device state store: one reference pipeline through
``Hypervisor(device="cuda")`` checked against host hashing, then p50 latency."""
import asyncio
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from agent_hypervisor_amd._native import C  # noqa: E402
from hypervisor import Hypervisor, SessionConfig  # noqa: E402
from hypervisor.audit.delta import SemanticDelta, VFSChange, delta_digest  # noqa: E402


async def one(hv):
    s = await hv.create_session(config=SessionConfig(enable_audit=True), creator_did="did:mesh:admin")
    sid = s.sso.session_id
    await hv.join_session(sid, "did:mesh:a", sigma_raw=0.8)
    await hv.activate_session(sid)
    ds = [s.delta_engine.capture("did:mesh:a", [VFSChange(path=f"/f{i}", operation="add", content_hash=f"h{i}")])
          for i in range(3)]
    saga = s.saga.create_saga(sid)
    step = s.saga.add_step(saga.saga_id, "action", "did:mesh:a", "/api/action")
    await s.saga.execute_step(saga.saga_id, step.step_id, executor=lambda: asyncio.sleep(0))
    root = await hv.terminate_session(sid)
    return s, ds, root


async def main():
    dev = sys.argv[1] if len(sys.argv) > 1 else "cuda"
    iters = int(sys.argv[2]) if len(sys.argv) > 2 else 2000
    t0 = time.perf_counter()
    hv = Hypervisor(device=dev)
    s, ds, root = await one(hv)
    print(f"first pipeline (incl. store init) {1e3 * (time.perf_counter() - t0):.1f} ms", flush=True)
    for d in ds:
        hd = SemanticDelta(d.delta_id, d.turn_id, d.session_id, d.agent_did, d.timestamp, d.changes, d.parent_hash)
        assert delta_digest(hd) == d.delta_hash, "device delta digest != host"
    assert C.merkle_root([d.delta_hash for d in ds]) == root, "device root != host"
    assert s.delta_engine.verify_chain()
    print("parity ok", root, flush=True)
    times = []
    for i in range(100 + iters):
        t0 = time.perf_counter_ns()
        await one(Hypervisor(device=dev))
        if i >= 100:
            times.append(time.perf_counter_ns() - t0)
    p50 = statistics.median(times) / 1e3
    out = {"device": dev, "p50_us": round(p50, 2), "mean_us": round(statistics.mean(times) / 1e3, 2),
           "p90_us": round(sorted(times)[int(0.9 * len(times))] / 1e3, 2), "info": hv._store.info()}
    print(json.dumps(out), flush=True)


if __name__ == "__main__" and (len(sys.argv) <= 3 or sys.argv[3] != "breakdown"):
    asyncio.run(main())


async def breakdown(dev: str = "cuda", iters: int = 1000, idle_us: int = 0) -> dict:
    """Median wall time of each API call of the reference pipeline."""
    import collections

    acc = collections.defaultdict(list)

    def tick(name, t0):
        acc[name].append(time.perf_counter_ns() - t0)
        return time.perf_counter_ns()

    for it in range(200 + iters):
        t = time.perf_counter_ns()
        hv = Hypervisor(device=dev)
        t = tick("hv_init", t)
        s = await hv.create_session(config=SessionConfig(enable_audit=True), creator_did="did:mesh:admin")
        sid = s.sso.session_id
        t = tick("create", t)
        await hv.join_session(sid, "did:mesh:a", sigma_raw=0.8)
        t = tick("join", t)
        await hv.activate_session(sid)
        t = tick("activate", t)
        for i in range(3):
            s.delta_engine.capture("did:mesh:a", [VFSChange(path=f"/f{i}", operation="add", content_hash=f"h{i}")])
            t = tick(f"capture{i}", t)
        saga = s.saga.create_saga(sid)
        t = tick("saga_create", t)
        step = s.saga.add_step(saga.saga_id, "action", "did:mesh:a", "/api/action")
        t = tick("add_step", t)
        await s.saga.execute_step(saga.saga_id, step.step_id, executor=lambda: asyncio.sleep(0))
        t = tick("execute_step", t)
        if idle_us:  # let the hash-engine wave drain first: terminate then measures its own work
            end = time.perf_counter_ns() + idle_us * 1000
            while time.perf_counter_ns() < end:
                pass
            t = tick("idle", t)
        await hv.terminate_session(sid)
        t = tick("terminate", t)
        if it < 200:
            acc.clear()
    return {k: round(statistics.median(v) / 1e3, 2) for k, v in acc.items()}


if __name__ == "__main__" and len(sys.argv) > 3 and sys.argv[3] == "breakdown":
    idle = int(sys.argv[4]) if len(sys.argv) > 4 else 0
    print(json.dumps(asyncio.run(breakdown(sys.argv[1], int(sys.argv[2]), idle))), flush=True)
