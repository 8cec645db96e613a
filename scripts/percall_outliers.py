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
import gc
_gc = {"n": 0, "ns": 0, "t0": 0}
def _gccb(phase, info):
    if info.get("generation") != 2:
        return
    if phase == "start":
        _gc["t0"] = time.perf_counter_ns()
    else:
        _gc["n"] += 1
        _gc["ns"] += time.perf_counter_ns() - _gc["t0"]
gc.callbacks.append(_gccb)
if os.environ.get("TUNE_GC"):
    from hypervisor.config import tune_gc
    tune_gc()
SLOW = {}  # wrapped callable -> [count over 1 ms, max µs]
def _wrap(obj, name, label):
    f = getattr(obj, name)
    def w(*a, **k):
        t0 = time.perf_counter_ns()
        try:
            return f(*a, **k)
        finally:
            dt = (time.perf_counter_ns() - t0) / 1e3
            if dt > 1000:
                e = SLOW.setdefault(label, [0, 0.0])
                e[0] += 1
                e[1] = max(e[1], round(dt, 1))
    setattr(obj, name, w)
if os.environ.get("WRAP", "1") == "1":
    for nm in ("alloc", "post_expect", "post", "verify_deferred", "capture", "call"):
        _wrap(st, nm, "store." + nm)
    _wrap(_device, "DeviceSession", "DeviceSession()")
    _wrap(_device, "session_views", "session_views")
    _wrap(_device, "SessionVFS", "SessionVFS()") if hasattr(_device, "SessionVFS") else None
    _wrap(_device._C, "uuid4", "_C.uuid4") if hasattr(_device, "_C") else None
def _launches():
    return st.info().get("launches", 0) if hasattr(st, "info") else 0
async def one():
    p = time.perf_counter_ns; t = {}
    a = p(); hv = Hypervisor(device=dev); t["init"] = p() - a
    a = p(); s = await hv.create_session(config=SessionConfig(enable_audit=True),
                                         creator_did="did:mesh:admin"); t["create"] = p() - a
    sid = s.sso.session_id
    a = p(); await hv.join_session(sid, "did:mesh:a", sigma_raw=0.8); t["join"] = p() - a
    a = p(); await hv.activate_session(sid); t["activate"] = p() - a
    a = p()
    for i in range(3):
        s.delta_engine.capture("did:mesh:a", [VFSChange(path=f"/f{i}", operation="add", content_hash=f"h{i}")])
    t["capture"] = p() - a
    a = p(); saga = s.saga.create_saga(sid); step = s.saga.add_step(saga.saga_id, "action", "did:mesh:a",
                                                                    "/api/action"); t["saga"] = p() - a
    a = p(); await s.saga.execute_step(saga.saga_id, step.step_id,
                                       executor=lambda: asyncio.sleep(0)); t["exec"] = p() - a
    a = p(); await hv.terminate_session(sid); t["term"] = p() - a
    a = p(); del s, hv, saga, step; t["teardown"] = p() - a
    return t
async def run(n):
    out = []
    for _ in range(n):
        i0 = st._c.info(); g0 = dict(st.grows); l0 = i0["launches"]; n0, ns0 = _gc["n"], _gc["ns"]
        lag0 = i0["posted"] - i0.get("worker_commands", i0["posted"])  # commands the worker has not run yet
        a = time.perf_counter_ns(); t = await one(); tot = time.perf_counter_ns() - a
        ev = {k: st.grows[k] - g0[k] for k in g0 if st.grows[k] != g0[k]}
        l1 = st._c.info()["launches"]
        if l1 != l0: ev["worker_launches"] = l1 - l0
        if _gc["n"] != n0: ev["gc2"] = (_gc["n"] - n0, round((_gc["ns"] - ns0) / 1e3, 1))
        ev["lag_before"] = lag0
        out.append((tot, t, ev))
    return out
asyncio.run(run(300))
res = asyncio.run(run(int(sys.argv[2]) if len(sys.argv) > 2 else 2000))
res.sort(key=lambda x: -x[0])
tots = sorted(r[0] for r in res)
print("p50", tots[len(tots)//2]/1e3, "p99", tots[int(.99*len(tots))]/1e3, "mean", sum(tots)/len(tots)/1e3)
lags = sorted(r[2]["lag_before"] for r in res)
print("worker lag before a pipeline (commands): p50", lags[len(lags) // 2], "p90", lags[int(.9 * len(lags))],
      "p99", lags[int(.99 * len(lags))], "max", lags[-1])
print("slow calls (>1 ms): count, max us", SLOW)
print("gen2 collections", _gc["n"], "total ms", round(_gc["ns"] / 1e6, 2), "worker launches", st._c.info()["launches"])
for tot, t, g in res[:12]:
    print(round(tot/1e3,1), {k: round(v/1e3,1) for k, v in t.items() if v > 20000}, g)
