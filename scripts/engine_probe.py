"""Hash-engine telemetry for the reference pipeline on the device store: per capture,
the engine's staging and hashing time (s_memrealtime, 10 ns ticks) and block count."""
import asyncio
import json
import statistics
import sys

sys.path.insert(0, ".")
from hypervisor import Hypervisor, SessionConfig  # noqa: E402
from hypervisor.audit.delta import VFSChange  # noqa: E402


async def main(n: int) -> dict:
    rows = {k: [] for k in range(3)}
    for it in range(n + 50):
        hv = Hypervisor(device="cuda")
        s = await hv.create_session(config=SessionConfig(enable_audit=True), creator_did="did:mesh:admin")
        sid = s.sso.session_id
        await hv.join_session(sid, "did:mesh:a", sigma_raw=0.8)
        await hv.activate_session(sid)
        ds = [s.delta_engine.capture("did:mesh:a", [VFSChange(path=f"/f{i}", operation="add", content_hash=f"h{i}")])
              for i in range(3)]
        saga = s.saga.create_saga(sid)
        step = s.saga.add_step(saga.saga_id, "action", "did:mesh:a", "/api/action")
        await s.saga.execute_step(saga.saga_id, step.step_id, executor=lambda: asyncio.sleep(0))
        await hv.terminate_session(sid)
        if it < 50:
            continue
        for k, d in enumerate(ds):
            r = hv._store.result(d._seq, 13)
            if r is not None:
                # result tuple k = result word k+1: words 10/11 stage/hash ticks, 12 blocks | batch << 32
                rows[k].append((r[9], r[10], r[11] & 0xFFFFFFFF, r[11] >> 32))
    out = {}
    for k, v in rows.items():
        if v:
            out[f"capture{k}"] = {"stage_us": statistics.median(x[0] for x in v) / 100,
                                  "hash_us": statistics.median(x[1] for x in v) / 100,
                                  "blocks": statistics.median(x[2] for x in v),
                                  "us_per_block": statistics.median(x[1] / max(1, x[2]) for x in v) / 100,
                                  "n": len(v)}
    return out


if __name__ == "__main__":
    print(json.dumps(asyncio.run(main(int(sys.argv[1]) if len(sys.argv) > 1 else 500))), flush=True)
