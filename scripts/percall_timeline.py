#!/usr/bin/env python3
"""Timeline of the per-call reference pipeline on the device store worker.

Runs the reference-harness pipeline (``benchmarks/bench_hypervisor.py:217-239``)
``ITERS`` times through ``Hypervisor(device="cuda")`` with the worker's timeline
trace on (``AHV_STORE_TRACE``), then prints, per command of the pipeline (median
over the pipelines), when the host posted it, when the worker picked it up and
finished it, and for captures when the hash engine hashed the record — all in µs
from the pipeline's first post.  Host and device clocks are aligned on the
earliest pickup (transit ≈ 0 for the fastest command).

    AHV_STORE_TRACE=65536 python scripts/percall_timeline.py
"""

from __future__ import annotations

import asyncio
import json
import os
import statistics
import sys
import time

os.environ.setdefault("AHV_STORE_TRACE", "65536")
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main() -> None:
    import numpy as np

    from hypervisor import Hypervisor, SessionConfig
    from hypervisor.audit.delta import VFSChange

    iters = int(os.environ.get("ITERS", "400"))
    dev = os.environ.get("DEV", "cuda")
    marks = []

    async def one():
        p = time.perf_counter_ns
        m = {"t0": p()}
        hv = Hypervisor(device=dev)
        st = hv._store
        m["q0"] = st._c.info()["posted"]
        s = await hv.create_session(config=SessionConfig(enable_audit=True), creator_did="did:mesh:admin")
        sid = s.sso.session_id
        await hv.join_session(sid, "did:mesh:a", sigma_raw=0.8)
        await hv.activate_session(sid)
        for i in range(3):
            s.delta_engine.capture("did:mesh:a", [VFSChange(path=f"/f{i}", operation="add", content_hash=f"h{i}")])
        saga = s.saga.create_saga(sid)
        step = s.saga.add_step(saga.saga_id, "action", "did:mesh:a", "/api/action")
        await s.saga.execute_step(saga.saga_id, step.step_id, executor=lambda: asyncio.sleep(0))
        m["t_term"] = p()
        await hv.terminate_session(sid)
        m["t_end"] = p()
        m["q1"] = st._c.info()["posted"]
        marks.append(m)
        return st

    async def run(n):
        st = None
        for _ in range(n):
            st = await one()
        return st

    asyncio.run(run(50))
    marks.clear()
    st = asyncio.run(run(iters))
    st.drain()
    tr = st._c.trace()
    if tr is None:
        raise SystemExit("tracing is off (AHV_STORE_TRACE)")
    cmd = np.frombuffer(tr[0], dtype=np.uint64).reshape(-1, 4).astype(np.int64)
    eng = np.frombuffer(tr[1], dtype=np.uint64).reshape(-1, 4).astype(np.int64)
    post = np.frombuffer(tr[2], dtype=np.uint64).astype(np.int64)
    tree = np.frombuffer(tr[3], dtype=np.uint64).reshape(-1, 4).astype(np.int64) if len(tr) > 3 else None
    helper = np.frombuffer(tr[4], dtype=np.uint64).reshape(-1, 4).astype(np.int64) if len(tr) > 4 else None
    cap = len(post)
    ok = cmd[:, 0] > 0
    seqs = cmd[ok, 0] - 1
    # clock alignment: device ticks are 10 ns; offset so that the fastest pickup has transit 0
    off = np.min(cmd[ok, 2] * 10 - post[seqs % cap])
    us = lambda ticks, base: (ticks * 10 - off - base) / 1e3  # noqa: E731
    per = []  # per pipeline: list of per-command dicts
    for m in marks:
        base = None
        rows_m = []
        for q in range(m["q0"], m["q1"]):
            c = cmd[q % cap]
            if c[0] != q + 1:
                continue
            pt = post[q % cap]
            if base is None:
                base = pt
            f = int(c[1])
            r = {"op": f & 0xFFFFFFFF, "post": (pt - base) / 1e3, "seen": us(c[2], base), "done": us(c[3], base),
                 "cmd_prefix_blocks": f >> 32 & 0xFF, "waited": (f >> 40 & 0xFFFFFF) / 100}
            e = eng[q % cap]
            if e[0] == q + 1:
                g = int(e[1])
                r.update(engine_start=us(e[2], base), engine_end=us(e[3], base), blocks=g & 0xFF, skip=g >> 8 & 0xFF,
                         batch=g >> 16 & 0xFF, stage_us=(g >> 24 & 0xFFFFF) / 100, hash_us=(g >> 44 & 0xFFFFF) / 100)
            if helper is not None and helper[q % cap][0] == q + 1:
                h = helper[q % cap]
                r.update(helper_start=us(h[2], base), helper_end=us(h[3], base), helper_mode=int(h[1]) & 0xFF,
                         helper_blocks=int(h[1]) >> 8 & 0xFF, helper_wave=int(h[1]) >> 16 & 0xFF)
            if tree is not None and tree[q % cap][0] == q + 1:
                t = tree[q % cap]
                r.update(tree_start=us(t[2], base), tree_end=us(t[3], base), tree_leaves=int(t[1]) & 0xFF,
                         tree_done=int(t[1]) >> 8 & 1, tree_cached=int(t[1]) >> 9 & 1)
            rows_m.append(r)
        m["term_host"] = (m["t_term"] - m["t0"]) / 1e3
        per.append(rows_m)
    from collections import Counter

    from agent_hypervisor_amd.models.store import OPS

    name = {v: k for k, v in OPS.items()}
    # pipelines interleave with the previous hypervisor's teardown commands: aggregate the
    # pipelines whose command sequence is the most common one
    sig = Counter(tuple(r["op"] for r in rm) for rm in per).most_common(1)[0][0]
    keep = [rm for rm in per if tuple(r["op"] for r in rm) == sig]
    med = lambda xs: round(statistics.median(xs), 2) if xs else None  # noqa: E731
    out = []
    for k, op in enumerate(sig):
        o = {"k": k, "op": name.get(op, op)}
        for f in ("post", "seen", "waited", "done", "cmd_prefix_blocks", "engine_start", "stage_us", "hash_us",
                  "engine_end", "blocks", "skip", "batch", "helper_start", "helper_end", "helper_mode",
                  "helper_blocks", "helper_wave", "tree_start", "tree_end", "tree_leaves", "tree_done", "tree_cached"):
            v = [rm[k][f] for rm in keep if f in rm[k]]
            if v:
                o[f] = med(v)
        out.append(o)
    print(json.dumps({"pipelines_with_this_sequence": len(keep), "of": len(per)}))
    lat = [(m["t_end"] - m["t0"]) / 1e3 for m in marks]
    print(json.dumps({"device": dev, "iters": iters, "p50_us": med(lat),
                      "terminate_called_us": med([m["term_host"] for m in marks]),
                      "spec_terminate": os.environ.get("AHV_SPEC_TERMINATE", "1")}))
    for o in out:
        print(json.dumps(o))


if __name__ == "__main__":
    main()
