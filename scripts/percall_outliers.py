#!/usr/bin/env python3
"""The slowest per-call reference pipelines and which API call made them slow
(``python scripts/percall_outliers.py cuda 3000``): p50 / p99 / mean, then the
eight slowest with every call over 20 µs and any table growth during them."""
import asyncio
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from hypervisor import Hypervisor, SessionConfig
from hypervisor.audit.delta import VFSChange
from hypervisor import _device
dev = sys.argv[1] if len(sys.argv) > 1 else "cpu"
st = _device._shared_store(dev)
rows = []
async def one():
    p = time.perf_counter_ns; t = {}
    a = p(); hv = Hypervisor(device=dev); t["init"] = p() - a
    a = p(); s = await hv.create_session(config=SessionConfig(enable_audit=True), creator_did="did:mesh:admin"); t["create"] = p() - a
    sid = s.sso.session_id
    a = p(); await hv.join_session(sid, "did:mesh:a", sigma_raw=0.8); t["join"] = p() - a
    a = p(); await hv.activate_session(sid); t["activate"] = p() - a
    a = p()
    for i in range(3):
        s.delta_engine.capture("did:mesh:a", [VFSChange(path=f"/f{i}", operation="add", content_hash=f"h{i}")])
    t["capture"] = p() - a
    a = p(); saga = s.saga.create_saga(sid); step = s.saga.add_step(saga.saga_id, "action", "did:mesh:a", "/api/action"); t["saga"] = p() - a
    a = p(); await s.saga.execute_step(saga.saga_id, step.step_id, executor=lambda: asyncio.sleep(0)); t["exec"] = p() - a
    a = p(); await hv.terminate_session(sid); t["term"] = p() - a
    a = p(); del s, hv, saga, step; t["teardown"] = p() - a
    return t
async def run(n):
    out = []
    for _ in range(n):
        g0 = dict(st.grows); a = time.perf_counter_ns(); t = await one(); tot = time.perf_counter_ns() - a
        out.append((tot, t, {k: st.grows[k] - g0[k] for k in g0 if st.grows[k] != g0[k]}))
    return out
asyncio.run(run(300))
res = asyncio.run(run(int(sys.argv[2]) if len(sys.argv) > 2 else 2000))
res.sort(key=lambda x: -x[0])
tots = sorted(r[0] for r in res)
print("p50", tots[len(tots)//2]/1e3, "p99", tots[int(.99*len(tots))]/1e3, "mean", sum(tots)/len(tots)/1e3)
for tot, t, g in res[:8]:
    print(round(tot/1e3,1), {k: round(v/1e3,1) for k, v in t.items() if v > 20000}, g)
