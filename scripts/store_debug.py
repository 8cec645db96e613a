import asyncio, hashlib, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from hypervisor import Hypervisor, SessionConfig
from hypervisor.audit.delta import SemanticDelta, VFSChange, canonical_payload

async def main():
    hv = Hypervisor(device=sys.argv[1] if len(sys.argv) > 1 else "cuda")
    s = await hv.create_session(config=SessionConfig(), creator_did="did:mesh:admin")
    sid = s.sso.session_id
    await hv.join_session(sid, "did:mesh:a", sigma_raw=0.8)
    for i in range(3):
        d = s.delta_engine.capture("did:mesh:a", [VFSChange(path=f"/f{i}", operation="add", content_hash=f"h{i}")])
        hd = SemanticDelta(d.delta_id, d.turn_id, d.session_id, d.agent_did, d.timestamp, d.changes, d.parent_hash)
        host = canonical_payload(hd)
        rec = d.record()
        print("turn", i + 1, "len", len(host), len(rec), "same bytes", host == rec)
        if host != rec:
            for k, (a, b) in enumerate(zip(host, rec)):
                if a != b:
                    print("  first diff at", k, host[max(0, k - 20):k + 20], rec[max(0, k - 20):k + 20])
                    break
        print("  device hash", d.device_hash())
        print("  sha(host)  ", hashlib.sha256(host).hexdigest())
        print("  sha(record)", hashlib.sha256(rec).hexdigest())

asyncio.run(main())
