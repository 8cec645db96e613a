"""K09 work-parallel Merkle (csrc/hip/merkle_tree.hip): one long chain reduced by
LDS subtrees per workgroup + multi-pass top, against the reference tree computed
independently on the host (hashlib for small chains, the SHA-NI level-wise
implementation for long ones)."""

from __future__ import annotations

import hashlib

import pytest
import torch

from agent_hypervisor_amd._native import C
from agent_hypervisor_amd.ops.audit import merkle_tree_root


def _leaves(n: int, seed: int = 0, device="cpu") -> torch.Tensor:
    g = torch.Generator().manual_seed(seed)
    return torch.randint(-(2**31), 2**31 - 1, (n, 8), generator=g, dtype=torch.int32).to(device)


def _hex(words) -> str:
    return "".join(f"{int(w) & 0xFFFFFFFF:08x}" for w in words)


def _reference(hexes: list[str]) -> str:
    level = list(hexes)
    while len(level) > 1:
        if len(level) % 2:
            level.append(level[-1])
        level = [hashlib.sha256((level[i] + level[i + 1]).encode()).hexdigest() for i in range(0, len(level), 2)]
    return level[0]


@pytest.mark.parametrize("n", [1, 2, 3, 5, 255, 256, 257, 511, 512, 513, 1025, 4097])
def test_tree_matches_reference_cpu_twin(n):
    lv = _leaves(n, seed=n)
    got = _hex(merkle_tree_root(lv).tolist())
    hexes = [_hex(r) for r in lv.tolist()]
    assert got == _reference(hexes) == C.merkle_root(hexes)
    assert got == C.merkle_root_words(lv.data_ptr(), n)


@pytest.mark.gpu
@pytest.mark.parametrize("n", [1, 255, 256, 257, 1_000_000, 16_000_000])
def test_tree_on_gfx950_matches_host(cuda_device, n):
    lv = _leaves(n, seed=7 + n)
    want = C.merkle_root_words(lv.data_ptr(), n) if n > 1 else _hex(lv[0].tolist())
    got = merkle_tree_root(lv.to(cuda_device))
    torch.cuda.synchronize()
    assert _hex(got.cpu().tolist()) == want
