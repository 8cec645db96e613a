"""Agent-sharded views (P02), overlapped collectives (P03) and session-row
migration (P08) — single-rank semantics plus a gloo world-2 run."""

from __future__ import annotations

import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from agent_hypervisor_amd.parallel import agent_shard as A


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("n,world", [(10, 3), (8, 4), (3, 5), (1000, 8)])
def test_owned_ranges_partition_and_owner_of(n, world):
    ranges = [A.owned_range(n, r, world) for r in range(world)]
    assert ranges[0][0] == 0 and ranges[-1][1] == n
    assert all(ranges[r][1] == ranges[r + 1][0] for r in range(world - 1))
    assert max(b - a for a, b in ranges) - min(b - a for a, b in ranges) <= 1
    for aid in range(n):
        r = A.owner_of(aid, n, world)
        assert ranges[r][0] <= aid < ranges[r][1]


def test_single_rank_paths():
    v = torch.arange(7, dtype=torch.float64)
    assert torch.equal(A.reduce_to_owners(v), v)
    oc = A.OverlappedCollective(torch.device("cpu"))
    t = torch.ones(3)
    oc.launch(lambda x: x.mul_(2), t).wait()
    assert t.tolist() == [2, 2, 2]


def _engine(seed=0):
    from agent_hypervisor_amd.models.engine import GovernanceEngine

    eng = GovernanceEngine(device="cpu", session_capacity=256, agent_capacity=512, seed=0x5EED0000 + seed)
    eng.register_synthetic_agents(128, seed=0)
    return eng


def test_export_import_rows_roundtrip():
    src, dst = _engine(0), _engine(1)
    batch = src.run_pipeline(32, deltas=2)
    slots = batch.slots().to(torch.int64)[:8]
    rows = A.export_rows(src, slots)
    packed, layout = A._pack(rows)
    back = A._unpack(packed, layout)
    assert all(torch.equal(back[k], rows[k]) for k in rows)
    new = A.import_rows(dst, back)
    for k in rows:
        assert torch.equal(getattr(dst.sessions, k).index_select(0, new.to(torch.int64)), rows[k])
    assert A._pack({k: v[:0] for k, v in rows.items()})[0].shape == (0, packed.shape[1])


def _worker(rank: int, world: int, port: int) -> None:
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        n = 11
        part = torch.arange(n, dtype=torch.float64) * (rank + 1)
        mine = A.reduce_to_owners(part)
        s, e = A.owned_range(n, rank, world)
        assert torch.equal(mine, torch.arange(s, e, dtype=torch.float64) * 3)
        # migrate rank r's first (r+1) sessions to the other rank
        eng = _engine(rank)
        batch = eng.run_pipeline(16, deltas=2)
        slots = batch.slots().to(torch.int64)
        other = 1 - rank
        per_dest = [None, None]
        per_dest[other] = A.export_rows(eng, slots[: rank + 1])
        per_dest[rank] = A.export_rows(eng, slots[:0])
        got = A.exchange_rows(per_dest)
        assert got[rank]["sess_state"].shape[0] == 0
        assert got[other]["sess_state"].shape[0] == other + 1
        sent = [None, None]
        dist.all_gather_object(sent, {k: v.tolist() for k, v in per_dest[other].items()})
        assert {k: v.tolist() for k, v in got[other].items()} == sent[other]
        A.import_rows(eng, got[other])
    finally:
        dist.destroy_process_group()


def test_agent_shard_gloo_world2():
    mp.start_processes(_worker, args=(2, _free_port()), nprocs=2, join=True, start_method="spawn")
