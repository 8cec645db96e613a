#!/usr/bin/env python3
"""Host cost of the store's native entry points one call at a time (not in bursts):
post, post_expect, verify_expects with nothing due, and the Python-level wrappers
the per-call API uses — to find where a speculated API call's microseconds go.
Prints one JSON object (median ns per call)."""

from __future__ import annotations

import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main() -> None:
    from agent_hypervisor_amd.models import store as S
    from hypervisor import _device

    dev = os.environ.get("DEV", "cuda")
    st = _device._shared_store(dev)
    c = st._c
    tok = (None, lambda a, r: RuntimeError("x"), 0)
    out = {}

    def timed(name, fn, n=2000, between=None):
        ts = []
        for _ in range(n):
            if between is not None:
                between()
            a = time.perf_counter_ns()
            fn()
            ts.append(time.perf_counter_ns() - a)
        out[name] = statistics.median(ts[n // 5:])

    drain = st.drain
    timed("post_nop_single", lambda: c.post(S.OP_NOP, [], None), between=drain)
    timed("post_nop_args7", lambda: c.post(S.OP_NOP, [1, 2, 3, 4, 5, 6, 7], None), between=drain)
    timed("post_expect_nop", lambda: c.post_expect(S.OP_NOP, [], None, (0,), tok), between=drain)
    timed("verify_expects_empty", lambda: c.verify_expects(False), between=lambda: (drain(), c.verify_expects(True)))
    timed("verify_deferred_empty", st.verify_deferred, between=lambda: (drain(), c.verify_expects(True)))

    def post_then_verify():
        c.post_expect(S.OP_NOP, [], None, (0,), tok)
        c.verify_expects(False)

    timed("post_expect_then_verify", post_then_verify, between=drain)
    # the pieces of a speculated activate_session
    import asyncio

    from hypervisor import Hypervisor, SessionConfig

    parts = {"guard": [], "activate_speculated": [], "activate_session": [], "join_session": []}

    async def one():
        hv = Hypervisor(device=dev)
        m = await hv.create_session(SessionConfig(enable_audit=True), "did:mesh:admin")
        sid = m.sso.session_id
        a = time.perf_counter_ns()
        await hv.join_session(sid, "did:mesh:a", sigma_raw=0.8)
        parts["join_session"].append(time.perf_counter_ns() - a)
        a = time.perf_counter_ns()
        m.sso._guard()
        parts["guard"].append(time.perf_counter_ns() - a)
        a = time.perf_counter_ns()
        m.sso._activate_speculated()
        parts["activate_speculated"].append(time.perf_counter_ns() - a)
        m2 = await hv.create_session(SessionConfig(enable_audit=True), "did:mesh:admin")
        await hv.join_session(m2.sso.session_id, "did:mesh:a", sigma_raw=0.8)
        a = time.perf_counter_ns()
        await hv.activate_session(m2.sso.session_id)
        parts["activate_session"].append(time.perf_counter_ns() - a)

    async def run():
        for _ in range(1500):
            await one()

    asyncio.run(run())
    for k, v in parts.items():
        out["api_" + k] = statistics.median(v[300:])
    t0 = time.perf_counter_ns()
    for _ in range(20000):
        time.perf_counter_ns()
    out["perf_counter_overhead"] = (time.perf_counter_ns() - t0) / 20000
    print(json.dumps({k: round(v, 1) for k, v in out.items()}))


if __name__ == "__main__":
    main()
