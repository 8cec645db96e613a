"""Device-authoritative state store (``Hypervisor(device=...)``) on its CPU twin.

The gfx950 worker and the CPU twin execute the same command processor
(``csrc/include/ahv/store.h``), so these tests pin the store's semantics to the
host engines without a GPU; ``tests/test_gpu_store.py`` repeats the parity
checks on the device.  The suites that re-express the reference's behaviour
(and the reference's own 326 tests, when mounted) are re-run with
``AHV_STORE=cpu`` so every public API call goes through the store.
"""

from __future__ import annotations

import asyncio
import os
import subprocess
import sys

import pytest

from agent_hypervisor_amd._native import C
from hypervisor import Hypervisor, SessionConfig
from hypervisor.audit.delta import SemanticDelta, VFSChange, delta_digest
from hypervisor.liability.vouching import VouchingError
from hypervisor.models import ExecutionRing, SessionState
from hypervisor.saga.state_machine import SagaState, StepState
from hypervisor.session import SessionLifecycleError, SessionParticipantError

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


async def _pipeline(hv):
    s = await hv.create_session(config=SessionConfig(enable_audit=True), creator_did="did:mesh:admin")
    sid = s.sso.session_id
    ring = await hv.join_session(sid, "did:mesh:a", sigma_raw=0.8)
    await hv.activate_session(sid)
    ds = [s.delta_engine.capture("did:mesh:a", [VFSChange(path=f"/f{i}", operation="add", content_hash=f"h{i}")])
          for i in range(3)]
    saga = s.saga.create_saga(sid)
    step = s.saga.add_step(saga.saga_id, "action", "did:mesh:a", "/api/action")
    await s.saga.execute_step(saga.saga_id, step.step_id, executor=lambda: asyncio.sleep(0))
    root = await hv.terminate_session(sid)
    return s, ring, ds, root, saga, step


def check_pipeline_parity(device: str) -> None:
    async def run():
        hv = Hypervisor(device=device)
        s, ring, ds, root, saga, step = await _pipeline(hv)
        assert ring is ExecutionRing.RING_2_STANDARD
        for d in ds:  # device digests == host canonical-JSON SHA-256 of the same fields
            hd = SemanticDelta(d.delta_id, d.turn_id, d.session_id, d.agent_did, d.timestamp, d.changes,
                               d.parent_hash)
            assert delta_digest(hd) == d.delta_hash
            assert d.record() == C.delta_payload(hd)
        assert ds[1].parent_hash == ds[0].delta_hash and ds[0].parent_hash is None
        assert root == C.merkle_root([d.delta_hash for d in ds])
        assert s.sso.state is SessionState.ARCHIVED
        assert step.state is StepState.COMMITTED and saga.state is SagaState.RUNNING
        assert s.delta_engine.verify_chain()
        c = hv.commitment.get_commitment(s.sso.session_id)
        assert c.merkle_root == root and c.delta_count == 3 and c.participant_dids == ["did:mesh:a"]
        ds[1].agent_did = "did:mesh:tampered"
        assert not s.delta_engine.verify_chain()

    asyncio.run(run())


def check_merkle_roots_track_chain(device: str) -> None:
    """compute_merkle_root / terminate after every capture (immediately, and after
    the hash engine has gone idle and precomputed its provisional root), with two
    sessions' captures interleaved and chains past the 64-leaf speculation limit:
    every root equals the host Merkle root of the digests so far."""
    import time

    async def run():
        hv = Hypervisor(device=device)
        a = await hv.create_session(SessionConfig(), creator_did="did:mesh:admin")
        b = await hv.create_session(SessionConfig(), creator_did="did:mesh:admin")
        for m in (a, b):
            await hv.join_session(m.sso.session_id, "did:mesh:x", sigma_raw=0.8)
            await hv.activate_session(m.sso.session_id)
        for i in range(70):
            for m in (a, b) if i % 3 else (b, a):
                m.delta_engine.capture("did:mesh:x", [VFSChange(path=f"/p{i}", operation="add", content_hash=f"c{i}")])
            if i % 5 == 0:
                time.sleep(0.0005)  # let the engine idle: the provisional root is ready
            m = a if i % 2 else b
            want = C.merkle_root([d.delta_hash for d in m.delta_engine.deltas])
            assert m.delta_engine.compute_merkle_root() == want, (i, device)
        for m in (a, b):
            want = C.merkle_root([d.delta_hash for d in m.delta_engine.deltas])
            assert await hv.terminate_session(m.sso.session_id) == want
        for n in range(1, 6):  # short chains terminated right after the last capture
            m = await hv.create_session(SessionConfig(), creator_did="did:mesh:admin")
            await hv.join_session(m.sso.session_id, "did:mesh:x", sigma_raw=0.8)
            await hv.activate_session(m.sso.session_id)
            for i in range(n):
                m.delta_engine.capture("did:mesh:x", [VFSChange(path=f"/q{i}", operation="add", content_hash=None)])
            if n % 2:
                time.sleep(0.0005)
            want = C.merkle_root([d.delta_hash for d in m.delta_engine.deltas])
            assert await hv.terminate_session(m.sso.session_id) == want

    asyncio.run(run())


def check_liability_parity(device: str) -> None:
    """Vouch / σ_eff / exposure / slash cascade on the store == the host engines."""

    async def run():
        hosts, devs = Hypervisor(device="host"), Hypervisor(device=device)
        out = []
        for hv in (hosts, devs):
            v, r = hv.vouching, []
            v.vouch("did:a", "did:b", "s1", 0.9, bond_pct=0.4)
            v.vouch("did:c", "did:b", "s1", 0.8, bond_pct=0.2)
            v.vouch("did:b", "did:d", "s1", 0.7)
            v.vouch("did:e", "did:a", "s1", 0.95, bond_pct=0.5)
            for bad in (("did:a", "did:a", 0.9), ("did:x", "did:y", 0.3), ("did:b", "did:a", 0.9)):
                with pytest.raises(VouchingError):
                    v.vouch(bad[0], bad[1], "s1", bad[2])
            with pytest.raises(VouchingError, match="exceed max exposure"):
                v.vouch("did:a", "did:z", "s1", 0.9, bond_pct=0.5)
            r.append(v.compute_sigma_eff("did:b", "s1", 0.3, 0.65))
            r.append(v.get_total_exposure("did:a", "s1"))
            scores = {"did:a": 0.9, "did:b": 0.4, "did:c": 0.8, "did:e": 0.95}
            res = hv.slashing.slash("did:b", "s1", 0.4, 0.95, "drift", scores)
            r.append([(c.voucher_did, c.sigma_before, c.sigma_after) for c in res.voucher_clips])
            r.append(sorted(scores.items()))
            r.append([(h.vouchee_did, h.cascade_depth, h.reason, len(h.voucher_clips)) for h in hv.slashing.history])
            r.append([x.is_active for x in v.records()])
            r.append(v.release_session_bonds("s1"))
            out.append(r)
        assert out[0] == out[1]

    asyncio.run(run())


def check_lifecycle_errors(device: str) -> None:
    async def run():
        hv = Hypervisor(device=device)
        s = await hv.create_session(SessionConfig(max_participants=2, min_sigma_eff=0.7), "did:admin")
        sid = s.sso.session_id
        with pytest.raises(SessionLifecycleError, match="no participants"):
            await hv.activate_session(sid)
        assert await hv.join_session(sid, "did:a", sigma_raw=0.96) is ExecutionRing.RING_2_STANDARD
        with pytest.raises(SessionParticipantError, match="already in session"):
            await hv.join_session(sid, "did:a", sigma_raw=0.9)
        assert await hv.join_session(sid, "did:b", sigma_raw=0.1) is ExecutionRing.RING_3_SANDBOX
        with pytest.raises(SessionParticipantError, match="capacity"):
            await hv.join_session(sid, "did:c", sigma_raw=0.9)
        s.sso.leave("did:b")
        assert [p.agent_did for p in s.sso.participants] == ["did:a"] and s.sso.participant_count == 1
        await hv.activate_session(sid)
        with pytest.raises(SessionLifecycleError, match="Allowed"):
            await hv.activate_session(sid)
        assert await hv.terminate_session(sid) is None  # no deltas → no root
        with pytest.raises(SessionLifecycleError):
            await hv.terminate_session(sid)
        assert s.sso.state is SessionState.ARCHIVED and s.sso.terminated_at is not None

    asyncio.run(run())


def check_saga_compensation(device: str) -> None:
    async def run():
        hv = Hypervisor(device=device)
        s = await hv.create_session(SessionConfig(), "did:admin")
        g = s.saga.create_saga(s.sso.session_id)
        a = s.saga.add_step(g.saga_id, "a", "did:x", "/a", undo_api="/undo_a")
        b = s.saga.add_step(g.saga_id, "b", "did:x", "/b")
        c = s.saga.add_step(g.saga_id, "c", "did:x", "/c", undo_api="/undo_c")
        for st in (a, b, c):
            await s.saga.execute_step(g.saga_id, st.step_id, executor=lambda: asyncio.sleep(0))

        async def comp(step):
            return "undone"

        failed = await s.saga.compensate(g.saga_id, comp)
        assert [f.step_id for f in failed] == [b.step_id]
        assert (a.state, b.state, c.state) == (StepState.COMPENSATED, StepState.COMPENSATION_FAILED,
                                               StepState.COMPENSATED)
        assert g.state is SagaState.ESCALATED and "1 step(s) failed compensation" in g.error
        assert g.to_dict()["steps"][1]["error"] == "No Undo_API available"

    asyncio.run(run())


def test_pipeline_parity_cpu_twin():
    check_pipeline_parity("cpu")


def test_merkle_roots_track_chain_cpu_twin():
    check_merkle_roots_track_chain("cpu")


def test_liability_parity_cpu_twin():
    check_liability_parity("cpu")


def test_lifecycle_errors_cpu_twin():
    check_lifecycle_errors("cpu")


def test_saga_compensation_cpu_twin():
    check_saga_compensation("cpu")


def test_default_mode_is_host_without_gpu():
    from hypervisor.config import store_mode

    import torch

    assert store_mode(None) in ("host", "cuda")
    assert store_mode("auto") == ("cuda" if torch.cuda.is_available() else "host")


def _run_suites(store: str, files: list[str]) -> None:
    env = dict(os.environ, AHV_STORE=store, PYTHONDONTWRITEBYTECODE="1")
    marks = ["-m", "not gpu"] if store == "cpu" else []
    p = subprocess.run([sys.executable, "-m", "pytest", "-q", "-x", "-p", "no:cacheprovider", *marks, *files],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=900)
    assert p.returncode == 0, p.stdout[-3000:] + p.stderr[-2000:]


PARITY_SUITES = [
    "tests/test_hv_integration.py", "tests/test_hv_liability.py", "tests/test_hv_rings.py",
    "tests/test_hv_saga.py", "tests/test_hv_services.py", "tests/test_hv_session.py", "tests/test_api.py",
    "tests/test_checkpoint.py", "tests/test_examples.py",
]


@pytest.mark.slow
def test_parity_suites_through_cpu_twin_store():
    _run_suites("cpu", PARITY_SUITES)


@pytest.mark.slow
@pytest.mark.skipif(not os.path.isdir("/root/reference/tests"), reason="reference checkout not mounted")
def test_reference_oracle_through_cpu_twin_store():
    env = {k: v for k, v in os.environ.items() if k != "PYTHONPATH"}
    env.update(PYTHONPATH=ROOT, PYTHONDONTWRITEBYTECODE="1", AHV_SKIP_AUTOBUILD="1", AHV_STORE="cpu")
    cmd = [sys.executable, "-m", "pytest", "/root/reference/tests", "-q", "-p",
           "agent_hypervisor_amd.utils.pytest_async",
           "-p", "no:cacheprovider", "-c", os.devnull, "--rootdir", "/tmp"]
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=900, env=env, cwd="/tmp")
    assert p.returncode == 0 and "326 passed" in p.stdout, p.stdout[-3000:]


@pytest.mark.parametrize("dev", ["cpu", pytest.param("cuda", marks=pytest.mark.gpu)])
def test_records_larger_than_the_hash_window_chain_correctly(dev):
    """A record past the worker's 16 KiB LDS window is hashed from the arena: the
    parent digest must be spliced there first (found by the store program fuzz in
    csrc/tests/host_selftest.cpp)."""
    import hashlib

    async def go():
        hv = Hypervisor(device=dev)
        s = await hv.create_session(config=SessionConfig(enable_audit=True), creator_did="did:mesh:admin")
        sid = s.sso.session_id
        await hv.join_session(sid, "did:mesh:a", sigma_raw=0.8)
        await hv.activate_session(sid)
        sizes = [10, 20000, 40, 17000]
        ds = [s.delta_engine.capture("did:mesh:a", [VFSChange(path=f"/f{i}", operation="add",
                                                              content_hash="x" * n)])
              for i, n in enumerate(sizes)]
        parent = None
        for d in ds:
            raw = d.record()
            assert len(raw) > 16384 or d.delta_hash
            assert d.parent_hash == parent
            assert d.delta_hash == hashlib.sha256(raw).hexdigest()
            parent = d.delta_hash
        assert s.delta_engine.verify_chain()
        assert hv.verify_audit([sid]).ok
        root = await hv.terminate_session(sid)
        assert root == C.merkle_root([d.delta_hash for d in ds])

    asyncio.run(go())
