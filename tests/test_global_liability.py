"""Agent-global liability kernels (K04 exposure, K06 slash stage, X02 sparse
apply) against plain-Python oracles of the reference formulas — on the CPU
twin here and on the gfx950 kernels in the GPU run."""

from __future__ import annotations

import pytest
import torch

from agent_hypervisor_amd.ops.global_liability import ResidentBonds
from agent_hypervisor_amd.parallel import collectives as X


def _oracle_exposure(b: ResidentBonds) -> list[float]:
    out = [0.0] * b.agents
    vr, bd, ac = b.voucher.tolist(), b.bonded.tolist(), b.active.tolist()
    for e in range(b.edges):  # creation order (edges are stored voucher-major, in order)
        if ac[e]:
            out[vr[e]] += bd[e]
    return out


def _run(dev: str) -> None:
    b = ResidentBonds(3000, 4, dev, seed=3)
    b.active[::7] = 0  # some bonds already released
    out = torch.zeros(b.agents, dtype=torch.float64, device=dev)
    b.exposure(out)
    assert out.cpu().tolist() == _oracle_exposure(b)  # exact: per-row creation-order sums

    ids = torch.tensor([5, 17, 17, 2999, 42], dtype=torch.int32, device=dev)
    active_before = b.active.cpu().clone()
    cap = 128
    pid = torch.full((cap,), -1, dtype=torch.int32, device=dev)
    pf = torch.ones(cap, dtype=torch.float64, device=dev)
    cur = torch.zeros(1, dtype=torch.int64, device=dev)
    b.slash_clip(ids, 0.95, pid, pf, cur)
    # oracle: every live incoming bond of a slashed vouchee is released once, its voucher clipped by (1-ω)
    vr, ve = b.voucher.tolist(), b.vouchee.tolist()
    want = sorted(vr[e] for e in range(b.edges) if ve[e] in {5, 17, 2999, 42} and active_before[e])
    n = int(cur.item())
    assert n == len(want)
    assert sorted(pid[:n].cpu().tolist()) == want and pid[n:].eq(-1).all()
    assert torch.all(pf[:n] == 1.0 - 0.95)
    for e in range(b.edges):
        if ve[e] in {5, 17, 2999, 42}:
            assert int(b.active[e]) == 0

    sigma = torch.rand(b.agents, dtype=torch.float64, generator=torch.Generator().manual_seed(1)).to(dev)
    ref = sigma.cpu().clone()
    for i, f in zip(pid[:n].cpu().tolist(), pf[:n].cpu().tolist()):
        ref[i] = max(ref[i].item() * f, 0.05)
    ref[ids.long().cpu()] = 0.0
    factor = torch.ones(b.agents, dtype=torch.float64, device=dev)
    X.merge_slash_fixed(sigma, ids, pid, pf, factor=factor)
    torch.testing.assert_close(sigma.cpu(), ref, rtol=1e-15, atol=0)
    assert torch.all(factor == 1.0)  # scratch left all-ones for the next step


def test_global_liability_cpu_twin():
    _run("cpu")


@pytest.mark.gpu
def test_global_liability_gfx950(cuda_device):
    _run("cuda")


def _run_storm(dev: str) -> None:
    """A larger storm: duplicate ids, in-degrees past the 8-edge unroll, a pair
    buffer smaller than the releases (the cursor still counts every one)."""
    g = torch.Generator().manual_seed(11)
    b = ResidentBonds(5000, 12, dev, seed=9)
    b.active[::5] = 0
    active_before = b.active.cpu().clone()
    ids = torch.randint(0, 5000, (1500,), generator=g, dtype=torch.int32)
    ids[::10] = ids[1::10]  # duplicates within the storm
    vr, ve = b.voucher.tolist(), b.vouchee.tolist()
    hit = set(ids.tolist())
    want = sorted(vr[e] for e in range(b.edges) if ve[e] in hit and active_before[e])
    for cap in (4 * len(want), len(want) // 3):
        bb = ResidentBonds(5000, 12, dev, seed=9)
        bb.active[::5] = 0
        pid = torch.full((cap,), -1, dtype=torch.int32, device=dev)
        pf = torch.ones(cap, dtype=torch.float64, device=dev)
        cur = torch.zeros(1, dtype=torch.int64, device=dev)
        bb.slash_clip(ids.to(dev), 0.9, pid, pf, cur)
        assert int(cur.item()) == len(want)
        got = sorted(x for x in pid.cpu().tolist() if x >= 0)
        if cap >= len(want):
            assert got == want
        else:
            assert len(got) == cap and not (set(got) - set(want))
        act = bb.active.cpu()
        assert all(int(act[e]) == 0 for e in range(bb.edges) if ve[e] in hit)


def test_slash_clip_storm_cpu_twin():
    _run_storm("cpu")


@pytest.mark.gpu
def test_slash_clip_storm_gfx950(cuda_device):
    _run_storm("cuda")
