"""§5.3 failure detection: fault injection in the kernel dispatcher is caught
by the audit layer, heartbeats expose a dead rank, collectives time out instead
of hanging, and a failed rank's sessions fail over to survivors from its last
checkpoint with their audit chains intact."""

from __future__ import annotations

import socket
import time
from datetime import timedelta

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from agent_hypervisor_amd.models.engine import GovernanceEngine
from agent_hypervisor_amd.ops import audit as A
from agent_hypervisor_amd.parallel.directory import SessionDirectory
from agent_hypervisor_amd.parallel.resilience import apply_failover, failover_plan, rehydrate
from agent_hypervisor_amd.runtime.checkpoint import CheckpointError, load_engine, save_engine, save_hypervisor
from agent_hypervisor_amd.utils.faults import inject


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


# ------------------------------------------------------------ fault injection


def test_corrupted_hash_batch_is_caught_by_verification():
    from hypervisor.audit.delta import DeltaEngine, VFSChange

    engines = []
    for s in range(8):
        de = DeltaEngine(f"session:{s}")
        for t in range(4):
            de.capture("did:a", [VFSChange(f"/f{t}", "add", f"h{t}")])
        engines.append(de)
    packed = A.pack_chains([de.deltas for de in engines])
    with inject("chain_hash", "corrupt", target="digest", index=37) as f:
        digests = A.chain_hashes(packed)
    assert f.hits == 1
    want = [d.delta_hash for de in engines for d in de.deltas]
    got = A.digests_to_hex(digests)
    assert sum(g != w for g, w in zip(got, want)) == 1  # exactly the corrupted record differs


def test_corrupted_pipeline_root_fails_checkpoint_verification(tmp_path):
    eng = GovernanceEngine(device="cpu", session_capacity=256, agent_capacity=256, seed=1)
    eng.register_synthetic_agents(100)
    eng.run_pipeline(64)
    with inject("pipeline", "corrupt", target="merkle_root", index=5) as f:
        eng.run_pipeline(64)
    assert f.hits == 1
    d = save_engine(eng, str(tmp_path / "e"))
    with pytest.raises(CheckpointError, match="re-verification"):
        load_engine(d, device="cpu")


def test_drop_and_delay_modes():
    t = torch.zeros(8, dtype=torch.float64)
    from agent_hypervisor_amd.ops import ledger as L

    with inject("drift", "drop") as f:
        sev = L.drift_severity(torch.full((8,), 0.9, dtype=torch.float64))
    assert f.hits == 1 and sev.numel() == 8  # launch skipped: outputs are whatever was allocated
    with inject("drift", "delay", seconds=0.05) as f:
        t0 = time.perf_counter()
        sev = L.drift_severity(torch.full((8,), 0.9, dtype=torch.float64))
        assert time.perf_counter() - t0 >= 0.05
    assert sev.tolist() == [4] * 8
    with pytest.raises(ValueError):
        inject("drift", "explode")
    del t


# ------------------------------------------------------------- failover plan


def test_failover_plan_rehomes_on_least_loaded():
    d = SessionDirectory(world=4)
    for k in range(20):
        d.place(f"s{k}")
    moves = failover_plan(d, [2])
    assert {s for s, f, _ in moves} == set(d.sessions_of(2)) and all(f == 2 for _, f, _ in moves)
    apply_failover(d, moves)
    assert d.load[2] == 0 and sum(d.load) == 20 and max(d.load) - min(d.load[:2] + d.load[3:]) <= 1
    with pytest.raises(RuntimeError):
        failover_plan(SessionDirectory(world=1), [0])


async def test_rehydrate_sessions_from_failed_rank_checkpoint(tmp_path):
    from hypervisor import Hypervisor, SessionConfig
    from hypervisor.audit.delta import VFSChange

    failed = Hypervisor()
    d = SessionDirectory(world=2)
    sids = []
    for k in range(4):
        m = await failed.create_session(SessionConfig(), "did:admin")
        sid = m.sso.session_id
        d._owner[sid] = 1
        d._load[1] += 1
        await failed.join_session(sid, f"did:a{k}", sigma_raw=0.8)
        await failed.activate_session(sid)
        for t in range(3):
            m.delta_engine.capture(f"did:a{k}", [VFSChange(f"/f{t}", "add", f"h{t}")])
        sids.append(sid)
    ck = save_hypervisor(failed, str(tmp_path / "rank1"))
    moves = failover_plan(d, [1])
    survivor = rehydrate(ck, moves, rank=0)
    apply_failover(d, moves)
    assert sorted(m.sso.session_id for m in survivor.sessions) == sorted(sids)
    m = survivor.get_session(sids[0])
    m.delta_engine.capture("did:a0", [VFSChange("/after-failover", "add", "x")])  # chain continues
    assert m.delta_engine.verify_chain() and d.owner(sids[0]) == 0


# ------------------------------------------------ heartbeats and timeouts


def _hb_worker(rank, world, port):
    from agent_hypervisor_amd.parallel.resilience import Heartbeat, guarded

    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world,
                            timeout=timedelta(seconds=20))
    hb = Heartbeat(interval_s=0.1).start()
    x = torch.ones(4)
    assert guarded(dist.all_reduce, x, timeout_s=10) and x.tolist() == [2.0] * 4
    dist.barrier()
    if rank == 1:
        hb.stop()  # rank 1 "dies": stops stamping and never joins the next collective
        store = dist.distributed_c10d._get_default_store()
        store.wait(["ahv/test/done"], timedelta(seconds=30))
    else:
        time.sleep(1.0)
        assert hb.dead_ranks(timeout_s=0.5) == [1]
        y = torch.ones(4)
        assert guarded(dist.all_reduce, y, timeout_s=1.0) is False  # times out instead of hanging
        hb.stop()
        dist.distributed_c10d._get_default_store().set("ahv/test/done", "1")


def test_heartbeat_detects_dead_rank_and_collective_times_out():
    mp.start_processes(_hb_worker, args=(2, _port()), nprocs=2, join=True, start_method="spawn")
