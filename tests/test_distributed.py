"""Session-sharded data parallelism on the CPU harness: the session directory
(P01/X07), every cross-rank collective X01–X09 under ``gloo`` with world size
2, sharded engines, and ``bench.py`` itself launched by ``torch.distributed.run``
(the same code path RCCL takes on MI355X)."""

from __future__ import annotations

import json
import os
import socket
import subprocess
import sys

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from agent_hypervisor_amd.parallel.directory import SessionDirectory, shard_counts, stable_rank

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


# ------------------------------------------------------------------ directory


class TestDirectory:
    def test_round_robin_and_idempotent(self):
        d = SessionDirectory(world=3)
        ranks = [d.place(f"s{k}") for k in range(7)]
        assert ranks == [0, 1, 2, 0, 1, 2, 0] and d.place("s0") == 0
        assert d.load == [3, 2, 2] and len(d) == 7 and d.is_local("s1", 1)

    def test_least_loaded(self):
        d = SessionDirectory(world=2, policy="least_loaded")
        d.place("a")
        d.place("b")
        d.release("a")
        assert d.place("c") == 0 and d.load == [1, 1]

    def test_hash_policy_is_stable(self):
        d1, d2 = SessionDirectory(world=8, policy="hash"), SessionDirectory(world=8, policy="hash")
        ids = [f"session:{k}" for k in range(100)]
        assert [d1.place(s) for s in ids] == [d2.place(s) for s in ids] == [stable_rank(s, 8) for s in ids]
        assert len(set(d1.place(s) for s in ids)) == 8

    def test_saga_routing(self):
        d = SessionDirectory(world=2)
        d.place("s0")
        d.place("s1")
        d.register_saga("g1", "s1")
        assert d.route_saga("g1") == (1, "s1") and d.route_saga("nope") is None
        with pytest.raises(KeyError):
            d.register_saga("g2", "unplaced")
        d.release("s1")
        assert d.route_saga("g1") is None and d.owner("s1") is None

    def test_rebalance(self):
        d = SessionDirectory(world=3, policy="hash")
        for k in range(30):
            d._owner[f"s{k}"] = 0
        d._load = [30, 0, 0]
        moves = d.rebalance_plan()
        d.apply(moves)
        assert d.load == [10, 10, 10] and len(moves) == 20
        with pytest.raises(ValueError):
            d.apply([(moves[0][0], 2, 1)] if d.owner(moves[0][0]) != 2 else [(moves[0][0], 0, 1)])

    def test_bad_args(self):
        with pytest.raises(ValueError):
            SessionDirectory(world=0)
        with pytest.raises(ValueError):
            SessionDirectory(world=2, policy="random")

    def test_shard_counts(self):
        assert shard_counts(10, 4) == [3, 3, 2, 2] and sum(shard_counts(100_003, 8)) == 100_003


# ---------------------------------------------------------------- collectives


def _collectives_worker(rank: int, world: int, port: int) -> None:
    from agent_hypervisor_amd.parallel import collectives as X

    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        assert X.world() == world
        # X04 counters
        st = torch.tensor([1, 2, 3, 4, 5, 6], dtype=torch.int64) * (rank + 1)
        assert X.allreduce_stats(st).tolist() == [3, 6, 9, 12, 15, 18]
        # X01 exposure
        e = torch.full((4,), 0.25 * (rank + 1), dtype=torch.float64)
        assert X.allreduce_exposure(e).tolist() == [0.75] * 4
        # X02 slash merge: rank0 clips agent0 by 0.5, rank1 clips agent0 by 0.5 and blacklists agent2
        sigma = torch.tensor([0.8, 0.9, 0.7], dtype=torch.float64)
        cf = torch.tensor([0.5, 1.0, 1.0], dtype=torch.float64)
        bl = torch.tensor([0, 0, rank], dtype=torch.uint8)
        out = X.merge_slash_effects(sigma, bl, cf)
        assert out.tolist() == [pytest.approx(0.2), 0.9, 0.0]
        # X02 sparse: the same clips as (id, factor) pairs, ragged across ranks
        ci = torch.tensor([0] if rank == 0 else [0, 1, 1], dtype=torch.int32)
        cfs = torch.tensor([0.5] if rank == 0 else [0.5, 0.9, 0.9], dtype=torch.float64)
        bli = torch.tensor([] if rank == 0 else [2], dtype=torch.int32)
        out = X.merge_slash_sparse(sigma, bli, ci, cfs)
        assert out.tolist() == [pytest.approx(0.2), pytest.approx(0.9 * 0.81), 0.0]
        # X03 deterministic risk
        r, c = X.allreduce_risk(torch.tensor([0.15, 0.6], dtype=torch.float64),
                                torch.tensor([1, 2], dtype=torch.int32))
        assert r.tolist() == [pytest.approx(0.3), 1.0] and c.tolist() == [2, 4]
        # X05 earliest ring: rank1 created the agent's session first
        ring = X.earliest_ring(torch.tensor([10 if rank == 0 else 3]), torch.tensor([2 if rank == 0 else 1]))
        assert ring.tolist() == [1]
        # X06 ragged commitments
        k = 2 + rank
        slots = torch.arange(k, dtype=torch.int64) + 100 * rank
        roots = torch.full((k, 8), rank, dtype=torch.int32)
        rk, sl, rt, ct = X.allgather_commitments(slots, roots, torch.full((k,), 3))
        assert rk.tolist() == [0, 0, 1, 1, 1] and sl.tolist() == [0, 1, 100, 101, 102]
        assert rt[:, 0].tolist() == [0, 0, 1, 1, 1] and ct.tolist() == [3] * 5
        # X08 broadcast
        ids = torch.tensor([5, 7, 9], dtype=torch.int32) if rank == 0 else torch.empty(0, dtype=torch.int32)
        assert X.broadcast_invalidations(ids).tolist() == [5, 7, 9]
        # X09 histograms
        assert X.reduce_histogram(torch.ones(8, dtype=torch.int64)).tolist() == [2] * 8
    finally:
        dist.destroy_process_group()


def _engine_worker(rank: int, world: int, port: int) -> None:
    from agent_hypervisor_amd.models.engine import GovernanceEngine
    from agent_hypervisor_amd.parallel import collectives as X

    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        eng = GovernanceEngine(device="cpu", session_capacity=512, agent_capacity=1024, seed=0x5EED0000 + rank)
        eng.register_synthetic_agents(256, seed=rank)
        stats = torch.zeros(6, dtype=torch.int64)
        batch = eng.run_pipeline(128, deltas=3, stats=stats)
        total = X.allreduce_stats(stats.clone())
        assert total[0].item() == 128 * world
        ok = int((batch.status() == 0).sum())
        assert total[1].item() == X.allreduce_stats(torch.tensor([ok] + [0] * 5))[0].item()
        # commitments of both shards gathered on every rank; ids never collide across ranks
        slots = batch.slots().to(torch.int64)
        rk, sl, rt, ct = X.allgather_commitments(slots, batch.roots(), torch.full((128,), 3))
        assert rk.numel() == 128 * world
        sid = [batch.session_id(i) for i in range(4)]
        gathered = [None] * world
        dist.all_gather_object(gathered, sid)
        assert len(set(sum(gathered, []))) == 4 * world
        # host re-verification of one materialised session on each shard
        m = batch.materialize(0)
        assert m.delta_engine.verify_chain()
    finally:
        dist.destroy_process_group()


def _spawn(fn, world=2):
    port = _free_port()
    mp.start_processes(fn, args=(world, port), nprocs=world, join=True, start_method="spawn")


def test_collectives_gloo_world2():
    _spawn(_collectives_worker)


def test_sharded_engines_gloo_world2():
    _spawn(_engine_worker)


def test_collectives_are_noops_single_rank():
    from agent_hypervisor_amd.parallel import collectives as X

    st = torch.arange(6)
    assert X.allreduce_stats(st) is st and X.world() == 1
    rk, sl, rt, ct = X.allgather_commitments(torch.arange(3), torch.zeros((3, 8), dtype=torch.int32), torch.ones(3))
    assert rk.tolist() == [0, 0, 0]


@pytest.mark.slow
@pytest.mark.parametrize("world", [2, 4, 8])
def test_bench_ranks_over_gloo(world):
    """The driver's scaling run (N = 1, 2, 4, 8 ranks of bench.py) rehearsed on the
    CPU: the same launcher, rank/env handling, double-buffered async X04
    all-reduce, max-over-ranks timing and the one JSON line from rank 0."""
    port = _free_port()
    env = dict(os.environ, OMP_NUM_THREADS="1", AHV_SKIP_AUTOBUILD="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(world),
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.join(ROOT, "bench.py"),
           "--gpus", str(world), "--device", "cpu", "--sessions", "256", "--agents", "2048", "--steps", "3",
           "--warmup", "1", "--no-scalar"]
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=900, env=env, cwd=ROOT)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1
    out = json.loads(lines[0])
    assert out["n_gpus"] == world and out["config"]["parallelism"] == f"dp{world}"
    assert out["config"]["global_batch"] == 256 * world
    assert out["last_step_counters"]["sessions"] == 256 * world and out["last_step_counters"]["ok"] == 256 * world
    assert out["value"] > 0 and out["steps"] == 3 and out["warmup"] == 1


@pytest.mark.parametrize("world", [2, 4])
def test_bench_self_launches_ranks(world):
    """``bench.py --gpus N`` with no launcher around it starts N rank processes by
    itself (the driver's scaling command is exactly this): the JSON line reports N
    ranks over the collective backend and N times the per-rank sessions."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env.update(OMP_NUM_THREADS="1", AHV_SKIP_AUTOBUILD="1")
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(world), "--device", "cpu",
           "--sessions", "256", "--agents", "2048", "--steps", "3", "--warmup", "1", "--no-scalar"]
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=600, env=env, cwd=ROOT)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1
    out = json.loads(lines[0])
    assert out["n_gpus"] == world and out["config"]["parallelism"] == f"dp{world}"
    assert out["collective_backend"] == "gloo" and out["launcher"].startswith("bench.py")
    assert out["last_step_counters"]["sessions"] == 256 * world


def test_bench_refuses_world_mismatch():
    """Under a launcher, ``WORLD_SIZE`` must equal ``--gpus`` (a silent 1-rank run
    reported as N GPUs is impossible)."""
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0", AHV_SKIP_AUTOBUILD="1")
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--device", "cpu",
           "--sessions", "64", "--agents", "256", "--steps", "1", "--warmup", "0", "--no-scalar"]
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=env, cwd=ROOT)
    assert p.returncode != 0 and "WORLD_SIZE=1 but --gpus 2" in p.stderr


def test_bench_launcher_reports_worst_rank_code():
    """A failing rank fails the whole self-launched run (its peers are stopped)."""
    import bench

    env_keep = dict(os.environ)
    try:
        os.environ.pop("WORLD_SIZE", None)
        code = bench.launch_ranks(2, ["--gpus", "2", "--device", "cpu", "--mix", "bogus"], grace_s=5.0)
    finally:
        os.environ.clear()
        os.environ.update(env_keep)
    assert code != 0


@pytest.mark.slow
def test_bench_hetero_mix_over_gloo():
    """``bench.py --mix hetero`` at 2 ranks on the CPU twin: each rank re-runs its
    packed heterogeneous batch every step over freed store rows, and the outcomes of
    every re-run equal the first run's (asserted inside bench.py)."""
    port = _free_port()
    env = dict(os.environ, OMP_NUM_THREADS="1", AHV_SKIP_AUTOBUILD="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.join(ROOT, "bench.py"),
           "--gpus", "2", "--device", "cpu", "--mix", "hetero", "--sessions", "1500", "--agents", "2048",
           "--steps", "2", "--warmup", "1", "--no-scalar"]
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=900, env=env, cwd=ROOT)
    assert p.returncode == 0, p.stderr[-3000:]
    out = json.loads([l for l in p.stdout.splitlines() if l.startswith("{")][-1])
    assert out["mix"] == "hetero" and out["config"]["model"] == "heterogeneous_governance_pipeline"
    assert out["last_step_counters"]["sessions"] == 3000 and 0 < out["last_step_counters"]["ok"] < 3000
    h = out["hetero"]
    assert h["sessions"] == 1500 and h["deltas"] > 1500 and 0 < h["committed_roots"] <= 1500
