"""The X01–X10 merge math over the in-process fake-rank world.

Same functions as the gloo (tests/test_distributed.py) and RCCL runs, at world
sizes up to 8 without spawning processes; the fake group reduces in rank order,
so every result is deterministic."""

from __future__ import annotations

import threading

import pytest
import torch

from agent_hypervisor_amd.parallel import collectives as X
from agent_hypervisor_amd.parallel.fake import FakeGroup, run_ranks


@pytest.mark.parametrize("world", [1, 2, 3, 8])
def test_counters_exposure_histograms(world):
    def body(rank):
        assert X.world() == world and X.rank() == rank
        st = X.allreduce_stats(torch.arange(6, dtype=torch.int64) * (rank + 1))
        e = X.allreduce_exposure(torch.full((3,), 0.5, dtype=torch.float64))
        h = X.reduce_histogram(torch.ones(4, dtype=torch.int64))
        return st.tolist(), e.tolist(), h.tolist()

    tri = world * (world + 1) // 2
    for st, e, h in run_ranks(world, body):
        assert st == [k * tri for k in range(6)]
        assert e == [0.5 * world] * 3
        assert h == [world] * 4


def _slash_inputs(world, A=64, seed=0):
    g = torch.Generator().manual_seed(seed)
    sigma = torch.rand(A, generator=g, dtype=torch.float64)
    per_rank = []
    for _ in range(world):
        k = int(torch.randint(0, 12, (1,), generator=g))
        ids = torch.randint(0, A, (k,), generator=g, dtype=torch.int32)
        om = torch.rand(k, generator=g, dtype=torch.float64) * 0.9
        bl = torch.randint(0, A, (int(torch.randint(0, 3, (1,), generator=g)),), generator=g, dtype=torch.int32)
        per_rank.append((ids, 1.0 - om, bl))
    return sigma, per_rank


def _sequential(sigma, per_rank, floor=0.05):
    """The documented cross-rank convention applied naively: every clip one at a
    time with its own floor (clips commute), then the blacklists (a blacklist
    from any rank zeroes the agent — no rank here reports a blacklist-then-clip
    floor outcome; that case is pinned by test_cycle_blacklist_then_clip_floor)."""
    s = sigma.clone()
    for ids, f, _ in per_rank:
        for i, x in zip(ids.tolist(), f.tolist()):
            s[i] = max(s[i].item() * x, floor)
    for _, _, bl in per_rank:
        s[bl.long()] = 0.0
    return s


@pytest.mark.parametrize("world", [1, 2, 4, 8])
def test_slash_merge_dense_and_sparse_match_sequential(world):
    sigma, per_rank = _slash_inputs(world, seed=world)
    want = _sequential(sigma, per_rank)

    def body(rank):
        ids, f, bl = per_rank[rank]
        cf = torch.ones_like(sigma)
        cf.index_reduce_(0, ids.long(), f, "prod")
        blv = torch.zeros(sigma.numel(), dtype=torch.uint8)
        blv[bl.long()] = 1
        dense = X.merge_slash_effects(sigma, blv, cf)
        sparse = X.merge_slash_sparse(sigma, bl, ids, f)
        return dense, sparse

    for dense, sparse in run_ranks(world, body):
        torch.testing.assert_close(sparse, dense, rtol=0, atol=0)
        torch.testing.assert_close(dense, want, rtol=1e-12, atol=1e-15)


def test_cycle_blacklist_then_clip_floor():
    """within one rank the reference blacklists the vouchee first and
    clips later, so an agent clipped after its own blacklist (vouch cycle) ends at
    the floor.  The merge reproduces SlashingEngine exactly on one rank, and a
    plain blacklist from another rank still wins."""
    from hypervisor.liability.slashing import SlashingEngine
    from hypervisor.liability.vouching import VouchingEngine

    ve = VouchingEngine()
    ve.vouch("did:a", "did:b", "s", 0.9, bond_pct=0.2)
    ve._creates_cycle = lambda *a: False  # force the cycle the admission check would reject
    ve.vouch("did:b", "did:a", "s", 0.9, bond_pct=0.2)
    scores = {"did:a": 0.0, "did:b": 0.5}
    SlashingEngine(ve).slash("did:b", "s", 0.5, 0.95, "x", scores)
    # A is clipped, wiped, cascaded (blacklisted → 0); B, blacklisted first, is clipped back to the floor
    assert scores["did:b"] == 0.05 and scores["did:a"] == 0.0

    ids = {"did:a": 0, "did:b": 1}
    sigma = torch.tensor([0.0, 0.5], dtype=torch.float64)
    bl, fl = torch.tensor([1, 0], dtype=torch.int32), torch.tensor([1], dtype=torch.int32)
    clip_ids = torch.tensor([ids["did:a"], ids["did:b"]], dtype=torch.int32)
    clip_f = torch.tensor([0.05, 0.05], dtype=torch.float64)
    got = run_ranks(1, lambda r: X.merge_slash_sparse(sigma, bl, clip_ids, clip_f, floored_ids=fl))[0]
    assert got.tolist() == [scores["did:a"], scores["did:b"]]
    cf = torch.ones(2, dtype=torch.float64)
    cf.index_reduce_(0, clip_ids.long(), clip_f, "prod")
    dense = run_ranks(1, lambda r: X.merge_slash_effects(sigma, torch.tensor([1, 1]), cf,
                                                         floored=torch.tensor([0, 1])))[0]
    assert dense.tolist() == got.tolist()

    def two(rank):  # rank 0 floored B, rank 1 blacklisted B outright → the lower outcome (0) wins
        if rank == 0:
            return X.merge_slash_sparse(sigma, bl, clip_ids, clip_f, floored_ids=fl)
        return X.merge_slash_sparse(sigma, bl, torch.empty(0, dtype=torch.int32), torch.empty(0, dtype=torch.float64))

    for out in run_ranks(2, two):
        assert out.tolist()[1] == 0.0


def test_merge_slash_fixed_matches_sparse():
    world = 3
    sigma, per_rank = _slash_inputs(world, seed=7)
    cap = 16

    def body(rank):
        ids, f, bl = per_rank[rank]
        pi = torch.full((cap,), -1, dtype=torch.int32)
        pf = torch.ones(cap, dtype=torch.float64)
        pi[: ids.numel()] = ids
        pf[: f.numel()] = f
        b = torch.full((4,), -1, dtype=torch.int32)
        b[: bl.numel()] = bl
        fixed = X.merge_slash_fixed(sigma.clone(), b, pi, pf)
        return fixed, X.merge_slash_sparse(sigma, bl, ids, f)

    for fixed, sparse in run_ranks(world, body):
        torch.testing.assert_close(fixed, sparse, rtol=0, atol=0)


def test_risk_is_rank_order_independent():
    parts = [torch.tensor([0.1 * (r + 1), 1e-9 * r, 0.3], dtype=torch.float64) for r in range(5)]

    def run(order):
        return run_ranks(5, lambda r: X.allreduce_risk(parts[order[r]]))[0]

    a = run([0, 1, 2, 3, 4])
    b = run([4, 2, 0, 3, 1])
    assert torch.equal(a, b)
    assert a.tolist()[2] == 1.0  # clamped after the sum


def test_earliest_ring_commitments_broadcast():
    world = 4

    def body(rank):
        ring = X.earliest_ring(torch.tensor([10 - rank]), torch.tensor([rank % 3]))
        k = rank + 1
        rk, sl, rt, ct = X.allgather_commitments(torch.arange(k, dtype=torch.int64) + 10 * rank,
                                                 torch.full((k, 8), rank, dtype=torch.int32), torch.full((k,), 2))
        ids = torch.tensor([4, 5], dtype=torch.int32) if rank == 1 else torch.empty(0, dtype=torch.int32)
        b = X.broadcast_invalidations(ids, src=1)
        return ring.tolist(), rk.tolist(), sl.tolist(), b.tolist()

    for ring, rk, sl, b in run_ranks(world, body):
        assert ring == [0]  # rank 3 created first (seq 7), ring 3 % 3 = 0
        assert rk == [0, 1, 1, 2, 2, 2, 3, 3, 3, 3]
        assert sl == [0, 10, 11, 20, 21, 22, 30, 31, 32, 33]
        assert b == [4, 5]


def test_failing_rank_does_not_deadlock():
    def body(rank):
        if rank == 2:
            raise RuntimeError("rank 2 lost")
        X.allreduce_stats(torch.zeros(6, dtype=torch.int64))
        return rank

    with pytest.raises(RuntimeError, match="rank 2 lost"):
        run_ranks(4, body)
    assert X.world() == 1  # the calling thread never had a fake group installed


def test_group_is_thread_local():
    g = FakeGroup(2)
    seen = []

    def other():
        seen.append(X.world())

    X.set_thread_group(g)
    g._local.rank = 0
    try:
        t = threading.Thread(target=other)
        t.start()
        t.join()
        assert X.world() == 2
    finally:
        X.set_thread_group(None)
    assert seen == [1]


def test_merge_slash_fixed_floored_codes_match_sparse():
    """Blacklist-then-clip (code 1 → floor) on one rank, plain blacklist (code 2 → 0)
    on another: the fixed-capacity path with codes equals the exact sparse merge."""
    world = 3
    sigma, per_rank = _slash_inputs(world, seed=11)
    cap = 16

    def body(rank):
        ids, f, bl = per_rank[rank]
        floored = bl[: max(1, bl.numel() // 2)] if rank != 1 else bl[:0]
        pi = torch.full((cap,), -1, dtype=torch.int32)
        pf = torch.ones(cap, dtype=torch.float64)
        pi[: ids.numel()] = ids
        pf[: f.numel()] = f
        b = torch.full((4,), -1, dtype=torch.int32)
        b[: bl.numel()] = bl
        codes = torch.full((4,), 2, dtype=torch.int32)
        codes[: bl.numel()] = torch.where(torch.isin(bl, floored), 1, 2).to(torch.int32)
        fixed = X.merge_slash_fixed(sigma.clone(), b, pi, pf, blacklist_codes=codes)
        return fixed, X.merge_slash_sparse(sigma, bl, ids, f, floored_ids=floored)

    outs = run_ranks(world, body)
    for fixed, sparse in outs:
        torch.testing.assert_close(fixed, sparse, rtol=0, atol=0)
    assert any(bool((o[1] == 0.05).any()) for o in outs)  # the floor case is exercised
