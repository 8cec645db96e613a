#!/usr/bin/env python3
"""Host CPU cost of each primitive on the per-call device path (ns per call,
median of bursts): the native transport calls, the id / row helpers, and the
Python API objects built around them — where the device path's host time goes
compared with the host engines (VERDICT r5 "What's weak" #1).

    DEV=cuda python scripts/probe_percall_costs.py
"""

from __future__ import annotations

import asyncio
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def bench(fn, n=2000, reps=15, setup=None, after=None) -> float:
    out = []
    for _ in range(reps):
        if setup is not None:
            setup()
        t0 = time.perf_counter_ns()
        for _ in range(n):
            fn()
        out.append((time.perf_counter_ns() - t0) / n)
        if after is not None:
            after()
    return round(statistics.median(out), 1)


def main() -> None:
    from agent_hypervisor_amd._native import C as _C
    from agent_hypervisor_amd.models import store as S
    from hypervisor import Hypervisor, SessionConfig
    from hypervisor import _device
    from hypervisor.audit.delta import VFSChange

    dev = os.environ.get("DEV", "cuda")
    st = _device._shared_store(dev)
    c = st._c
    out = {"device": dev}
    drain = st.drain
    out["py_noop_call"] = bench(lambda: None)
    out["pybind_n_expects"] = bench(c.n_expects)
    out["post_nop"] = bench(lambda: c.post(S.OP_NOP, [], None), n=200, after=drain)
    out["post_nop_3args"] = bench(lambda: c.post(S.OP_NOP, [1, 2, 3], None), n=200, after=drain)
    tok = (None, None, None)
    out["post_expect_nop"] = bench(lambda: c.post_expect(S.OP_NOP, [1, 2, 3], None, (0,), tok), n=200,
                                   after=lambda: (st.verify_deferred(True), drain()))
    out["verify_expects_empty"] = bench(lambda: c.verify_expects(False))
    out["store_verify_deferred_empty"] = bench(st.verify_deferred)
    out["try_result_done"] = bench(lambda: c.try_result(0, 2, 0) if False else None)
    q = c.post(S.OP_NOP, [], None)
    c.keep(q)
    drain()
    out["try_result_ready"] = bench(lambda: c.try_result(q, 2, 0))
    out["uuid4_id"] = bench(lambda: _C.uuid4_id("session:"))
    out["uuid4"] = bench(lambda: _C.uuid4("saga:"))
    rows = []
    out["alloc_S"] = bench(lambda: rows.append(st.alloc("S")), n=500,
                           after=lambda: (st.release_many("S", rows), rows.clear(), st.reclaim("S")))
    out["agent_id"] = bench(lambda: st.agent_id("did:mesh:a"))
    out["now_us"] = bench(_device._now_us)
    out["dbits"] = bench(lambda: S.dbits(0.8))
    out["join_predict"] = bench(lambda: _C.join_predict(1, False, 0, 10, 0.8, 0.5, True))

    # API objects (host side only, no command)
    out["Hypervisor_init_close"] = bench(lambda: Hypervisor(device=dev).close(), n=500)
    out["Hypervisor_init_host"] = bench(lambda: Hypervisor(), n=500)

    async def pipe(d):
        hv = Hypervisor(device=d)
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

    async def many(d, n):
        await asyncio.gather(*[pipe(d) for _ in range(n)])

    for d in (dev, "host"):
        asyncio.run(many(d, 500))
        ts = []
        for _ in range(5):
            t0 = time.process_time_ns()
            asyncio.run(many(d, 2000))
            ts.append((time.process_time_ns() - t0) / 2000)
        out[f"gather_cpu_ns_per_pipeline_{d}"] = round(statistics.median(ts), 1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
