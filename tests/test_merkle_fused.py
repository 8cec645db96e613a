"""K09 with the leaf gather and the root scatter fused (``merkle_roots(leaf_idx=,
root_out=, root_row=, gate=)``) equals gather → K09 → masked scatter."""

from __future__ import annotations

import pytest
import torch

from agent_hypervisor_amd.ops import audit as A


def _case(dev: str) -> None:
    g = torch.Generator().manual_seed(7)
    table = torch.randint(-2**31, 2**31 - 1, (500, 8), generator=g, dtype=torch.int64).to(torch.int32)
    lens = torch.randint(0, 9, (60,), generator=g)
    offs = torch.cat([torch.zeros(1, dtype=torch.int64), lens.cumsum(0)]).to(torch.int32)
    idx = torch.randint(0, 500, (int(lens.sum()),), generator=g, dtype=torch.int64)
    rows = torch.randperm(200, generator=g)[:60].to(torch.int64)
    gate = (torch.rand(200, generator=g) < 0.7).to(torch.int64)
    ref = A.merkle_roots(offs, table.index_select(0, idx))
    want = torch.full((200, 8), 5, dtype=torch.int32)
    want[rows] = torch.where(gate[rows, None] != 0, ref, torch.zeros_like(ref))
    t, o, i, r, gt = (x.to(dev) for x in (table, offs, idx, rows, gate))
    out = torch.full((200, 8), 5, dtype=torch.int32, device=dev)
    A.merkle_roots(o, t, leaf_idx=i, root_out=out, root_row=r, gate=gt)
    assert torch.equal(out.cpu(), want)
    plain = A.merkle_roots(o, t, leaf_idx=i)
    assert torch.equal(plain.cpu(), ref)


def test_fused_merkle_host():
    _case("cpu")


@pytest.mark.gpu
def test_fused_merkle_gfx950():
    _case("cuda")
