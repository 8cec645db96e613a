"""Hash-engine throughput of the device store: N captures posted back to back, then
one compute_merkle_root (which drains the engine).  The slope over N is the
engine's per-delta cost (staging + serial SHA-256); the intercept is transport
plus the tree."""
import asyncio
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from hypervisor import Hypervisor, SessionConfig  # noqa: E402
from hypervisor.audit.delta import VFSChange  # noqa: E402


async def one(hv, n):
    s = await hv.create_session(config=SessionConfig(enable_audit=True), creator_did="did:mesh:admin")
    await hv.join_session(s.sso.session_id, "did:mesh:a", sigma_raw=0.8)
    await hv.activate_session(s.sso.session_id)
    t0 = time.perf_counter_ns()
    for i in range(n):
        s.delta_engine.capture("did:mesh:a", [VFSChange(path=f"/f{i}", operation="add", content_hash=f"h{i}")])
    t1 = time.perf_counter_ns()
    s.delta_engine.compute_merkle_root()
    t2 = time.perf_counter_ns()
    return (t1 - t0) / 1e3, (t2 - t0) / 1e3


async def main():
    dev = sys.argv[1] if len(sys.argv) > 1 else "cuda"
    out = {}
    hv = Hypervisor(device=dev)
    for n in (1, 2, 3, 6, 12, 24):
        post, total = [], []
        for it in range(300):
            p, t = await one(hv, n)
            if it >= 50:
                post.append(p)
                total.append(t)
        out[n] = {"post_us": round(statistics.median(post), 2), "total_us": round(statistics.median(total), 2)}
    print(json.dumps(out), flush=True)


asyncio.run(main())
