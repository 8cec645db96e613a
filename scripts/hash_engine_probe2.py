"""Per-capture hash-engine telemetry (result-slot words 10-12: staging ticks,
hashing ticks at 100 MHz, blocks) for the reference pipeline's 3 captures."""
import asyncio
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from hypervisor import Hypervisor, SessionConfig  # noqa: E402
from hypervisor.audit.delta import VFSChange  # noqa: E402


async def main():
    hv = Hypervisor(device=sys.argv[1] if len(sys.argv) > 1 else "cuda")
    rows = {0: [], 1: [], 2: []}
    for it in range(300):
        s = await hv.create_session(config=SessionConfig(enable_audit=True), creator_did="did:mesh:admin")
        await hv.join_session(s.sso.session_id, "did:mesh:a", sigma_raw=0.8)
        await hv.activate_session(s.sso.session_id)
        ds = [s.delta_engine.capture("did:mesh:a", [VFSChange(path=f"/f{i}", operation="add", content_hash=f"h{i}")])
              for i in range(3)]
        s.delta_engine.compute_merkle_root()
        for i, d in enumerate(ds):
            r = hv._store.result(d._seq, 12)  # tuple index i = slot word i + 1
            if it >= 50 and r is not None:
                rows[i].append((r[9] * 10 / 1e3, r[10] * 10 / 1e3, r[11], d._plen))
    out = {i: {"stage_us": round(statistics.median(x[0] for x in v), 2),
               "hash_us": round(statistics.median(x[1] for x in v), 2),
               "blocks": v[0][2], "bytes": v[0][3]} for i, v in rows.items() if v}
    print(json.dumps(out), flush=True)


asyncio.run(main())
