"""Stress: per-call sessions with 1-8 captures each, awaited terminates; counts device
roots that differ from the host's prediction (and chains whose device digests differ
from hashlib over the canonical payload).  Worker features via AHV_STORE_* env."""
import asyncio
import hashlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from hypervisor import Hypervisor, SessionConfig  # noqa: E402
from hypervisor.audit.delta import VFSChange, canonical_payload  # noqa: E402
from agent_hypervisor_amd.models.store import StoreError  # noqa: E402


def _around(b: bytes, at):
    """The bytes around offset ``at`` (None: no difference)."""
    if at is None:
        return None
    return b[max(0, at - 8):at + 24].decode("latin1")


async def main(n: int, dev: str) -> dict:
    hv = Hypervisor(device=dev)
    bad_root = bad_digest = 0
    detail = []
    for k in range(n):
        m = await hv.create_session(SessionConfig(), creator_did="did:mesh:admin")
        sid = m.sso.session_id
        await hv.join_session(sid, f"did:mesh:a{k % 7}", sigma_raw=0.8)
        await hv.activate_session(sid)
        for i in range(1 + k % 8):
            m.delta_engine.capture(f"did:mesh:a{k % 7}", [VFSChange(path=f"/f{i}", operation="add",
                                                                     content_hash=f"h{k}.{i}" * (1 + k % 5))])
        try:
            await hv.terminate_session(sid)
        except StoreError:
            bad_root += 1
        ds = m.delta_engine.deltas
        for i, d in enumerate(ds):
            raw = canonical_payload(d)
            if hashlib.sha256(raw).hexdigest() != d.delta_hash:
                bad_digest += 1
                rec = d.record()
                ok_rec = hashlib.sha256(rec).hexdigest() == d.delta_hash
                diff = next((j for j in range(min(len(rec), len(raw))) if rec[j] != raw[j]), None)
                detail.append({"k": k, "i": i, "n": len(ds), "len": len(raw), "rec_len": len(rec),
                               "arena_record_equals_render": rec == raw, "digest_of_arena_record": ok_rec,
                               "first_diff": diff, "hole": raw.find(b'"parent_hash": ') + 15,
                               "host_off": d._poff, "host_len": d._plen,
                               "dev_rows": {k: int(v[0]) for k, v in hv._store.gather(
                                   {"d_off": [d._didx], "d_len": [d._didx], "d_hole": [d._didx],
                                    "d_turn": [d._didx]}).items()},
                               "rec_at_diff": _around(rec, diff), "raw_at_diff": _around(raw, diff)})
                break
    return {"sessions": n, "bad_root": bad_root, "bad_digest_chains": bad_digest, "detail": detail[:5]}


if __name__ == "__main__":
    res = asyncio.run(main(int(sys.argv[1]) if len(sys.argv) > 1 else 2000,
                           sys.argv[2] if len(sys.argv) > 2 else "cuda"))
    res.update({k: v for k, v in os.environ.items() if k.startswith("AHV_STORE_")})
    print(json.dumps(res))
