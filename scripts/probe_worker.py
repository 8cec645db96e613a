#!/usr/bin/env python3
"""Micro-probes of the resident store worker (where a per-call pipeline's device
time goes): host post cost, NOP round trip, per-opcode round trips, and the hash
engine's own telemetry per capture (stage / hash time, blocks)."""

from __future__ import annotations

import asyncio
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main() -> None:
    from agent_hypervisor_amd.models import store as S
    from hypervisor import Hypervisor, SessionConfig
    from hypervisor import _device
    from hypervisor.audit.delta import VFSChange

    dev = os.environ.get("DEV", "cuda")
    st = _device._shared_store(dev)
    out = {}
    # host cost of a post (no wait), then the drain
    for _ in range(2000):
        st.post(S.OP_NOP, [])
    st.drain()
    # bursts well under the ring size: the post itself, never a wait for a free slot
    burst, posts = 256, []
    for _ in range(40):
        t0 = time.perf_counter_ns()
        for _ in range(burst):
            st.post(S.OP_NOP, [])
        posts.append((time.perf_counter_ns() - t0) / burst)
        st.drain()
    out["post_ns"] = statistics.median(posts)
    # a run far past the ring size: the worker's NOP throughput
    n = 20000
    t0 = time.perf_counter_ns()
    for _ in range(n):
        st.post(S.OP_NOP, [])
    st.drain()
    out["nop_throughput_ns"] = (time.perf_counter_ns() - t0) / n
    # round trips
    rt = []
    for _ in range(3000):
        a = time.perf_counter_ns()
        st.call(S.OP_NOP, [], 1)
        rt.append(time.perf_counter_ns() - a)
    out["nop_roundtrip_p50_us"] = statistics.median(rt[500:]) / 1e3

    # per-capture engine telemetry over reference pipelines
    stage, hashed, blocks, caps = [], [], [], []

    async def one():
        hv = Hypervisor(device=dev)
        s = await hv.create_session(config=SessionConfig(enable_audit=True), creator_did="did:mesh:admin")
        sid = s.sso.session_id
        await hv.join_session(sid, "did:mesh:a", sigma_raw=0.8)
        await hv.activate_session(sid)
        ds = [s.delta_engine.capture("did:mesh:a", [VFSChange(path=f"/f{i}", operation="add", content_hash=f"h{i}")])
              for i in range(3)]
        for d in ds:
            r = st.result(d._seq, 13)
            if r is not None and not r[0]:
                stage.append(r[9] / 100.0)
                hashed.append(r[10] / 100.0)
                blocks.append(r[11] & 0xFFFFFFFF)
                caps.append(d._plen)
        t = time.perf_counter_ns()
        await hv.terminate_session(sid)
        return time.perf_counter_ns() - t

    async def run():
        w = []
        for _ in range(400):
            w.append(await one())
        return w

    waits = asyncio.run(run())
    out["capture_stage_us_p50"] = statistics.median(stage[100:]) if stage else None
    out["capture_hash_us_p50"] = statistics.median(hashed[100:]) if hashed else None
    out["capture_blocks_p50"] = statistics.median(blocks[100:]) if blocks else None
    out["record_bytes_p50"] = statistics.median(caps[100:]) if caps else None
    out["terminate_us_p50"] = statistics.median(waits[100:]) / 1e3
    info = st.info()
    out["worker_busy_us_per_command"] = info.get("worker_busy_us", 0) / max(1, info.get("worker_commands", 1))
    out["engine_busy_us_per_job"] = info.get("engine_busy_us", 0) / max(1, info.get("engine_jobs", 1))
    print(json.dumps(out))


if __name__ == "__main__":
    main()
