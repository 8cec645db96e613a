"""gfx950 template pipeline over store rows (GovernanceEngine's ring) vs its host
twin: every session column and every canonical-JSON record byte-equal."""

from __future__ import annotations

import pytest
import torch

from agent_hypervisor_amd.models.engine import GovernanceEngine
from agent_hypervisor_amd.models.engine import EngineSessions as SessionTable

pytestmark = pytest.mark.gpu

NOW = 1767225600123456


def _pair(n_agents=300, cap=8192, seed=11, dids=None, sig=None):
    d = GovernanceEngine(device="cuda:0", session_capacity=cap, agent_capacity=max(n_agents, 8), seed=seed)
    h = GovernanceEngine(device="cpu", session_capacity=cap, agent_capacity=max(n_agents, 8), seed=seed)
    for e in (d, h):
        if dids is None:
            e.register_synthetic_agents(n_agents, seed=3)
        else:
            e.register_agents(dids, sig)
    return d, h


def _assert_tables_equal(d, h, bd, bh):
    sd, sh = bd.slots().cpu(), bh.slots()
    for col in SessionTable.COLUMNS:
        a = getattr(d.sessions, col).cpu().index_select(0, sd)
        b = getattr(h.sessions, col).index_select(0, sh)
        assert torch.equal(a, b), f"column {col} differs"
    for i in range(0, bd.n, max(1, bd.n // 37)):  # the records in the arena, byte for byte
        for k in range(int(h.sessions.delta_count[int(sh[i])])):
            assert bd.record(i, k) == bh.record(i, k), (i, k)


def test_pipeline_device_equals_host(cuda_device):
    d, h = _pair()
    agents = torch.randint(0, 300, (3000,), dtype=torch.int32, generator=torch.Generator().manual_seed(0))
    stats = torch.zeros(6, dtype=torch.int64, device=cuda_device)
    bd = d.run_pipeline(3000, agents=agents.to(cuda_device), now_us=NOW, stats=stats)
    bh = h.run_pipeline(3000, agents=agents, now_us=NOW)
    torch.cuda.synchronize()
    _assert_tables_equal(d, h, bd, bh)
    assert stats.tolist() == [3000, 3000, 3000, 9000, 3000, 3000]


def test_pipeline_skewed_lengths_device(cuda_device):
    """Lanes of one wave with very different message lengths exercise the
    non-uniform (urgent) compression path of the LDS ring."""
    dids = ["did:a", "did:mesh:" + "q" * 400, "did:" + "ü" * 50, 'did:"esc\\aped"\n', "did:mesh:mid-length-agent"]
    d, h = _pair(dids=dids, sig=[0.1, 0.61, 0.95, 0.6, 0.99], cap=1024)
    agents = torch.arange(640, dtype=torch.int32) % 5
    bd = d.run_pipeline(640, agents=agents.to(cuda_device), now_us=NOW, changes=[("/p/{i}" + "x" * 90, "add", "h{i}")])
    bh = h.run_pipeline(640, agents=agents, now_us=NOW, changes=[("/p/{i}" + "x" * 90, "add", "h{i}")])
    torch.cuda.synchronize()
    _assert_tables_equal(d, h, bd, bh)


@pytest.mark.parametrize("deltas", [1, 2, 5, 8])
def test_pipeline_delta_counts_device(cuda_device, deltas):
    d, h = _pair(cap=512)
    bd = d.run_pipeline(200, deltas=deltas, now_us=NOW + 999)
    bh = h.run_pipeline(200, deltas=deltas, now_us=NOW + 999)
    torch.cuda.synchronize()
    _assert_tables_equal(d, h, bd, bh)


def test_pipeline_materialized_roots_verify(cuda_device):
    d, _ = _pair(cap=256)
    b = d.run_pipeline(64, now_us=NOW)
    torch.cuda.synchronize()
    for i in range(0, 64, 7):
        m = b.materialize(i)
        assert m.delta_engine.verify_chain()
        assert m.delta_engine.compute_merkle_root() == b.merkle_root_hex(i)


def test_pipeline_large_batch_runs(cuda_device):
    eng = GovernanceEngine(device="cuda:0", session_capacity=1 << 18, agent_capacity=1 << 16, seed=1)
    eng.register_synthetic_agents(1 << 16)
    stats = torch.zeros(6, dtype=torch.int64, device=cuda_device)
    eng.run_pipeline(1 << 18, stats=stats)
    torch.cuda.synchronize()
    assert stats[0].item() == 1 << 18 and stats[1].item() == 1 << 18


_ADV = list('abcXYZ019:/-_. "\\{}') + ["\n", "\t", "\x00", "\x7f", "é", "中", "\U0001F600", "\ud800"]


def _adv_text(rng, lo, hi):
    return "".join(rng.choice(_ADV) for _ in range(rng.randint(lo, hi)))


@pytest.mark.parametrize("case", range(6))
def test_pipeline_adversarial_text_device(cuda_device, case):
    """Random DIDs (1–200 characters: JSON escapes, astral characters, lone
    surrogates), 0–3 change objects with long or null fields, 1–8 deltas and
    whole-second timestamps: every lane's message has its own byte phase and
    length (1–20+ SHA blocks, many window passes).  The host twin these are
    compared with is pinned to the reference package byte for byte by
    tests/test_differential_reference.py."""
    import random

    rng = random.Random(100 + case)
    dids = list(dict.fromkeys(_adv_text(rng, 1, 200) for _ in range(64)))
    specs = []
    for _ in range(rng.randint(0, 3)):
        p = _adv_text(rng, 0, 120).replace("{", "{{").replace("}", "}}") + "{i}"
        o = _adv_text(rng, 1, 8).replace("{", "{{").replace("}", "}}")
        hsh = None if rng.random() < 0.3 else _adv_text(rng, 0, 70).replace("{", "{{").replace("}", "}}")
        specs.append((p, o, hsh))
    deltas = rng.randint(1, 8)
    now = 1_767_225_600_000_000 - 2 if case % 2 else NOW
    d, h = _pair(dids=dids, sig=[0.9] * len(dids), cap=2048)
    n = 640
    agents = torch.randint(0, len(dids), (n,), dtype=torch.int32, generator=torch.Generator().manual_seed(case))
    bd = d.run_pipeline(n, agents=agents.to(cuda_device), deltas=deltas, now_us=now, changes=specs or None)
    bh = h.run_pipeline(n, agents=agents, deltas=deltas, now_us=now, changes=specs or None)
    torch.cuda.synchronize()
    _assert_tables_equal(d, h, bd, bh)


def test_pipeline_gc_retention_device(cuda_device):
    """GC retention from timestamps (retention shorter than the session): device rows
    equal the host twin's."""
    d, h = _pair()
    for e in (d, h):
        e.gc_retention_us = 4
    agents = torch.randint(0, 300, (3000,), dtype=torch.int32, generator=torch.Generator().manual_seed(5))
    bd = d.run_pipeline(3000, agents=agents.to(cuda_device), now_us=NOW)
    bh = h.run_pipeline(3000, agents=agents, now_us=NOW)
    torch.cuda.synchronize()
    _assert_tables_equal(d, h, bd, bh)
    assert bool((h.sessions.gc_retained[bh.slots()] == 2).all())
