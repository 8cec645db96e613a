#!/usr/bin/env python3
"""Median time of each public-API call of the reference pipeline (per-call API),
for one device: ``python scripts/percall_split.py cuda|cpu|host``."""
import asyncio
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from hypervisor import Hypervisor, SessionConfig
from hypervisor.audit.delta import VFSChange
dev = sys.argv[1] if len(sys.argv) > 1 else "cpu"
T = {}
def rec(k, dt): T.setdefault(k, []).append(dt)
async def one():
    p = time.perf_counter_ns
    a = p(); hv = Hypervisor(device=dev); rec("hv_init", p() - a)
    a = p(); s = await hv.create_session(config=SessionConfig(enable_audit=True),
                                         creator_did="did:mesh:admin"); rec("create", p() - a)
    sid = s.sso.session_id
    a = p(); await hv.join_session(sid, "did:mesh:a", sigma_raw=0.8); rec("join", p() - a)
    a = p(); await hv.activate_session(sid); rec("activate", p() - a)
    a = p()
    for i in range(3):
        s.delta_engine.capture("did:mesh:a", [VFSChange(path=f"/f{i}", operation="add", content_hash=f"h{i}")])
    rec("capture x3", p() - a)
    a = p(); saga = s.saga.create_saga(sid); rec("create_saga", p() - a)
    a = p(); step = s.saga.add_step(saga.saga_id, "action", "did:mesh:a", "/api/action"); rec("add_step", p() - a)
    a = p(); await s.saga.execute_step(saga.saga_id, step.step_id,
                                       executor=lambda: asyncio.sleep(0)); rec("execute_step", p() - a)
    a = p(); await hv.terminate_session(sid); rec("terminate", p() - a)
    a = p(); del s, hv, saga, step; rec("teardown", p() - a)
async def run(n):
    for _ in range(n): await one()
asyncio.run(run(500)); T.clear(); asyncio.run(run(3000))
tot = 0
for k, v in T.items():
    m = statistics.median(v) / 1e3; tot += m
    print(f"{k:14s} {m:7.2f} us")
print(f"{'sum':14s} {tot:7.2f} us")
