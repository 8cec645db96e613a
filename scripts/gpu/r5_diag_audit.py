"""Diagnose the batched-audit vs scalar mismatch on device-backed sessions (GPU)."""
import hashlib
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from test_audit_verify import _build, _scalar_bad_chains  # noqa: E402

from hypervisor.audit.delta import canonical_payload  # noqa: E402

dev = sys.argv[1] if len(sys.argv) > 1 else "cuda"
if len(sys.argv) > 2:  # first what the suite's preceding test does: thousands of concurrent pipelines
    import asyncio

    sys.path.insert(0, os.path.join(ROOT, "benchmarks"))
    from bench_api import reference_pipeline

    async def go(n):
        return await asyncio.gather(*[reference_pipeline(dev) for _ in range(n)])

    asyncio.run(go(int(sys.argv[2])))
hv = _build(300, deltas=4, device=dev)
ms = hv.sessions
tam = [3, 77, 150]
for k in tam:
    ms[k].delta_engine._deltas[0].turn_id += 1
rep = hv.verify_audit(device="cuda" if "cuda" in str(hv._store.device) else "cpu")
print("batched", len(rep.bad_chains), "scalar", len(_scalar_bad_chains(hv)))
for k in tam:
    m = ms[k]
    ds = m.delta_engine.deltas
    d0 = ds[0]
    raw = canonical_payload(d0)
    print(k, m.sso.session_id in rep.bad_chains, "dirty", [d.__dict__.get("_dirty") for d in ds],
          "stored", d0.delta_hash[:16], "recomputed",
          hashlib.sha256(raw.encode() if isinstance(raw, str) else raw).hexdigest()[:16],
          "turn", d0.turn_id, "n", len(ds), "seq", d0._seq, "didx", d0._didx,
          "dev_hash", (d0.__dict__.get("_dev_hash") or "")[:16], "res", hv._store.result(d0._seq, 9) is not None)
