"""Batched audit verification (hypervisor/audit/batch_verify.py): K10 chains, K09
roots vs commitments, K11 VFS contents vs their edit log, K12 goal hashes — the
batched answer must equal the scalar engines' answer (DeltaEngine.verify_chain,
compute_merkle_root, hashlib) on clean and on tampered state."""

from __future__ import annotations

import asyncio
import hashlib
import json
import os

import pytest
import torch

from hypervisor import Hypervisor, SessionConfig
from hypervisor.audit.batch_verify import verify_audit
from hypervisor.audit.delta import VFSChange
from hypervisor.saga.checkpoint import CheckpointManager


def _build(n: int, deltas: int = 3, device=None, terminate_every: int = 2) -> Hypervisor:
    hv = Hypervisor(device=device)

    async def go():
        for k in range(n):
            m = await hv.create_session(SessionConfig(), creator_did="did:mesh:admin")
            sid = m.sso.session_id
            await hv.join_session(sid, f"did:mesh:a{k % 7}", sigma_raw=0.8)
            await hv.activate_session(sid)
            for i in range(deltas + k % 3):
                m.sso.vfs.write(f"/f{i}", f"content {k}/{i} é", f"did:mesh:a{k % 7}")
                m.delta_engine.capture(f"did:mesh:a{k % 7}",
                                       [VFSChange(path=f"/f{i}", operation="add", content_hash=f"h{k}.{i}")])
            if k % 4 == 1:
                m.sso.vfs.write("/f0", "rewritten", f"did:mesh:a{k % 7}")
            if k % terminate_every == 0:
                await hv.terminate_session(sid)

    asyncio.run(go())
    return hv


def _scalar_bad_chains(hv) -> list[str]:
    return [m.sso.session_id for m in hv.sessions if not m.delta_engine.verify_chain()]


def test_clean_state_verifies_host():
    hv = _build(12)
    rep = hv.verify_audit(device="cpu")
    assert rep.ok, rep.to_dict()
    assert rep.sessions == 12 and rep.deltas == sum(len(m.delta_engine.deltas) for m in hv.sessions)
    assert rep.roots_checked == 6 and rep.files > 12


def test_tampering_is_found_and_matches_scalar_engines():
    hv = _build(10)
    ms = hv.sessions
    # K10: a payload field changed after hashing (stored hash no longer matches)
    ms[1].delta_engine._deltas[1].agent_did = "did:mesh:mallory"
    # K10: a broken parent link
    ms[3].delta_engine._deltas[2].parent_hash = "f" * 64
    # K09: a commitment whose root does not cover the chain
    rec = hv.commitment.get_commitment(ms[4].sso.session_id)
    rec.merkle_root = "0" * 63 + "1"
    # K11: a VFS file rewritten without an edit record
    ms[5].sso.vfs._files[ms[5].sso.vfs._resolve("/f1")] = "forged"
    rep = hv.verify_audit(device="cpu")
    assert sorted(rep.bad_chains) == sorted(_scalar_bad_chains(hv)) == sorted([ms[1].sso.session_id,
                                                                               ms[3].sso.session_id])
    assert rep.bad_roots == [ms[4].sso.session_id]
    assert rep.bad_files == [(ms[5].sso.session_id, ms[5].sso.vfs._resolve("/f1"))]
    assert not rep.ok


def test_snapshot_restore_and_delete_are_not_false_positives():
    hv = _build(2)
    vfs = hv.sessions[1].sso.vfs  # session 0 was terminated (its VFS garbage-collected)
    snap = vfs.create_snapshot()
    vfs.write("/f0", "changed after snapshot", "did:mesh:a1")
    vfs.restore_snapshot(snap, "did:mesh:a1")
    vfs.delete("/f1", "did:mesh:a1")
    assert hv.verify_audit(device="cpu").ok


def test_checkpoint_manager_goal_hashes():
    mgr = CheckpointManager()
    for s in range(20):
        mgr.save(f"saga:{s % 3}", f"step:{s}", f"goal number {s} ✓", {"k": s})
    assert mgr.verify("cpu") == []
    recs = mgr.export_records()
    back = CheckpointManager.from_records(json.loads(json.dumps(recs)), device="cpu")
    assert back.total_checkpoints == 20 and back.is_achieved("saga:1", "goal number 4 ✓", "step:4")
    recs[7]["goal_description"] = "a different goal"
    with pytest.raises(ValueError, match=recs[7]["checkpoint_id"]):
        CheckpointManager.from_records(recs, device="cpu")
    rep = verify_audit((), device="cpu", checkpoints=[mgr])
    assert rep.ok and rep.checkpoints == 20


def test_checkpoint_restore_uses_batched_verification(tmp_path):
    from agent_hypervisor_amd.runtime.checkpoint import CheckpointError, load_hypervisor, save_hypervisor

    hv = _build(6)
    d = save_hypervisor(hv, str(tmp_path / "ck"))
    back = load_hypervisor(d)
    assert len(back.sessions) == 6
    assert [e.content_hash for e in back.sessions[2].sso.vfs.edit_log] == \
        [e.content_hash for e in hv.sessions[2].sso.vfs.edit_log]
    assert back.verify_audit(device="cpu").ok
    # a VFS file altered on disk (its manifest digest re-signed) is caught by K11
    p = os.path.join(d, "sessions.jsonl")
    lines = open(p).read().splitlines()
    rec = json.loads(lines[3])
    path = next(iter(rec["vfs"]["files"]))
    rec["vfs"]["files"][path] = "tampered on disk"
    lines[3] = json.dumps(rec, sort_keys=True)
    open(p, "w").write("\n".join(lines) + "\n")
    from agent_hypervisor_amd.runtime import checkpoint as ck

    mp = os.path.join(d, "manifest.json")
    man = json.load(open(mp))
    man["files"]["sessions.jsonl"] = ck._sha(p)
    json.dump(man, open(mp, "w"))
    with pytest.raises(CheckpointError, match="does not match its logged content hash"):
        load_hypervisor(d)


def test_device_store_twin_sessions_verify():
    hv = _build(5, device="cpu")  # device-authoritative store, CPU twin
    rep = hv.verify_audit(device="cpu")
    assert rep.ok and rep.deltas > 0 and rep.roots_checked == 3


def test_rest_route(tmp_path):
    from fastapi.testclient import TestClient

    from hypervisor.api.server import create_app

    hv = _build(3)
    with TestClient(create_app(hv)) as c:
        body = c.get("/api/v1/audit/verify", params={"device": "cpu"}).json()
        assert body["ok"] and body["sessions"] == 3
        one = c.get("/api/v1/audit/verify", params={"device": "cpu", "session_id": hv.sessions[0].sso.session_id})
        assert one.json()["sessions"] == 1
        assert c.get("/api/v1/audit/verify", params={"session_id": "nope"}).status_code == 404


@pytest.mark.gpu
def test_gpu_batched_audit_matches_host_twin():
    hv = _build(300, deltas=4)
    ms = hv.sessions
    for k in (3, 77, 150):
        ms[k].delta_engine._deltas[0].turn_id += 1
    ms[10].sso.vfs._files[ms[10].sso.vfs._resolve("/f2")] = "x"
    mgr = CheckpointManager()
    for s in range(500):
        mgr.save(f"saga:{s % 9}", f"step:{s}", f"goal {s}")
    mgr._checkpoints["saga:4"][0].goal_hash = "0" * 16
    gpu = hv.verify_audit(device="cuda", checkpoints=[mgr])
    cpu = hv.verify_audit(device="cpu", checkpoints=[mgr])
    assert gpu.device.startswith("cuda")
    assert gpu.to_dict() | {"device": ""} == cpu.to_dict() | {"device": ""}
    from hypervisor.audit.delta import canonical_payload

    detail = [(ms[k].sso.session_id, ms[k].sso.session_id in gpu.bad_chains,
               [d.__dict__.get("_dirty") for d in ms[k].delta_engine.deltas],
               ms[k].delta_engine.deltas[0].delta_hash,
               hashlib.sha256(canonical_payload(ms[k].delta_engine.deltas[0])).hexdigest())
              for k in (3, 77, 150)]
    assert sorted(gpu.bad_chains) == sorted(_scalar_bad_chains(hv)), detail
    assert len(gpu.bad_files) == 1 and len(gpu.bad_checkpoints) == 1
    h = hashlib.sha256("x".encode()).hexdigest()
    assert h not in {e.content_hash for e in ms[10].sso.vfs.edit_log}
    assert torch.cuda.is_available()
