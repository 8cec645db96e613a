"""The template pipeline over store rows (csrc/hip/store_template.hip): one device
state for the headline path and ``Hypervisor.pipeline_batch``.

Every session the kernel writes must be an ordinary session of the hypervisor: its
records in the arena hash to its digests (scalar renderer + SHA-256), its root is
the reference Merkle root, ``verify_audit`` passes over the arena in place with
nothing staged, later lifecycle calls give the reference errors, and checkpoints
include it."""

from __future__ import annotations

import asyncio
import hashlib

import numpy as np
import pytest
import torch

from agent_hypervisor_amd.models import store_template as TT
from hypervisor import Hypervisor
from hypervisor.session import SessionLifecycleError

DEVICES = ["cpu", pytest.param("cuda", marks=pytest.mark.gpu)]


def _merkle(leaves: list[str]) -> str:
    level = list(leaves)
    while len(level) > 1:
        if len(level) % 2:
            level.append(level[-1])
        level = [hashlib.sha256((level[k] + level[k + 1]).encode()).hexdigest() for k in range(0, len(level), 2)]
    return level[0]


def _reference_records(sid: str, did: str, t0: int, deltas: int) -> list[bytes]:
    """The records the scalar API renders for the same deltas (reference delta.py:41-64)."""
    from hypervisor._clock import from_us
    from hypervisor.audit.delta import SemanticDelta, VFSChange, _payload_json

    out, parent = [], None
    for k in range(deltas):
        d = SemanticDelta(delta_id=f"delta:{k + 1}", turn_id=k + 1, session_id=sid, agent_did=did,
                          timestamp=from_us(t0 + 1 + k),
                          changes=[VFSChange(path=f"/f{k}", operation="add", content_hash=f"h{k}")],
                          parent_hash=parent)
        raw = _payload_json(d).encode()
        out.append(raw)
        parent = hashlib.sha256(raw).hexdigest()
    return out


@pytest.mark.parametrize("dev", DEVICES)
def test_template_batch_sessions_are_ordinary_store_sessions(dev):
    async def go():
        hv = Hypervisor(device=dev)
        st = hv._store
        agents = TT.AgentSet(st, [f"did:mesh:tmpl-agent-{k}" for k in range(7)] + ["did:x"],
                             [0.8, 0.3, 0.61, 0.96, 0.6, 0.95, 0.05, 0.7])
        n = 70
        run = TT.run(hv, n, agents=agents, session_agent=np.arange(n) % agents.count, now_us=1767225600123456)
        assert run.ok == n
        t0 = 1767225600123456
        for i in (0, 1, 5, 7, 69):
            sid = run.session_ids[i]
            m = hv.get_session(sid)
            did = agents.dids[i % agents.count]
            assert m.sso.state.value == "archived"
            ps = m.sso._participants
            assert list(ps) == [did]
            assert ps[did].sigma_raw == float(agents.sigma[i % agents.count])
            recs = _reference_records(sid, did, t0, 3)
            ds = m.delta_engine.deltas
            assert [d.record() for d in ds] == recs
            hashes = [hashlib.sha256(r).hexdigest() for r in recs]
            assert [d.delta_hash for d in ds] == hashes
            assert run.roots[sid] == _merkle(hashes)
            assert m.delta_engine.compute_merkle_root() == _merkle(hashes)
            assert m.delta_engine.verify_chain()
            g = m.saga.sagas[0]
            assert g.state.value == "running" and g.steps[0].state.value == "committed"
            with pytest.raises(SessionLifecycleError):
                await hv.terminate_session(sid)
        # audit over the arena in place: nothing rendered, nothing staged
        staged = []
        orig = st.stage
        st.stage = lambda data: staged.append(len(data)) or orig(data)
        try:
            rep = hv.verify_audit([s for s in run.session_ids[10:40]])
        finally:
            st.stage = orig
        assert rep.ok and rep.deltas == 90 and rep.roots_checked == 30, rep
        assert sum(staged) <= 30 * 3 * 4 + 4096  # row-index lists only, no payload bytes
        snaps = hv.snapshots()
        assert sum(1 for x in snaps if x.state.value == "archived") >= n
        return True

    assert asyncio.run(go())


@pytest.mark.parametrize("dev", DEVICES)
def test_template_rows_reset_and_rerun(dev):
    """The bench's steady state: rows freed in place and the whole pipeline re-run;
    counters match, new ids each launch, and a live row is never overwritten."""
    hv = Hypervisor(device=dev)
    st = hv._store
    agents = TT.AgentSet.synthetic(st, 256, seed=3, prefix="did:mesh:rerun-agent-")
    tp = TT.TemplatePipeline(st, 200, agents)
    stats = torch.zeros(6, dtype=torch.int64, device=st.device)
    sa = torch.randint(0, 256, (200,), dtype=torch.int32)
    b0, _ = tp.launch(sa, stats=stats)
    st0 = tp.tens["status"].clone()
    # without a reset every row is live: nothing is written
    tp.launch(sa, stats=stats)
    assert bool((tp.tens["status"] == 1).all())
    tp.reset()
    b2, _ = tp.launch(sa, stats=stats)
    assert torch.equal(tp.tens["status"], st0) and bool((st0 == 0).all())
    assert b2 == b0 + 400 and tp.session_ids(b0)[0] != tp.session_ids(b2)[0]
    other = TT.TemplatePipeline(st, 8, agents)  # another batch on the same store: its own id range
    b3, _ = other.launch(sa[:8])
    assert b3 >= b2 + 200
    got = stats.cpu().tolist()
    assert got == [600, 400, 400, 1200, 400, 400], got
    # the second run's rows carry the second run's ids
    words = st.gather({"s_uuid": (tp.slots[:1].astype(np.int64) * 4 + np.arange(4))})["s_uuid"]
    hexs = "".join(f"{int(w) & 0xFFFFFFFF:08x}" for w in words)
    assert tp.session_ids(b2)[0].replace("-", "").endswith(hexs)


@pytest.mark.parametrize("dev", DEVICES)
def test_pipeline_batch_routes_to_the_store(dev):
    hv = Hypervisor(device=dev)
    run = hv.pipeline_batch(64)
    assert run.ok == 64 and len(run.roots) == 64
    sid = run.session_ids[3]
    m = hv.get_session(sid)
    assert m.sso.session_id == sid and m.delta_engine.turn_count == 3
    assert m.delta_engine.verify_chain()


def test_pipeline_batch_needs_a_device_backed_hypervisor():
    with pytest.raises(RuntimeError, match="device-backed"):
        Hypervisor(device="host").pipeline_batch(4)


def test_template_checkpoint_round_trip(tmp_path):
    from agent_hypervisor_amd.runtime.checkpoint import load_hypervisor, save_hypervisor

    hv = Hypervisor(device="cpu")
    run = hv.pipeline_batch(20)
    d = save_hypervisor(hv, str(tmp_path / "ck"))
    hv2 = load_hypervisor(d, hv=Hypervisor(device="cpu"))
    for sid in run.session_ids[:5]:
        m = hv2.get_session(sid)
        assert m.delta_engine.compute_merkle_root() == run.roots[sid]
