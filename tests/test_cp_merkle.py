"""P06/X10: context-parallel Merkle roots equal the serial reference tree for
every chain length and rank count (odd-duplication edge cases included)."""

from __future__ import annotations

import hashlib
import socket

import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from agent_hypervisor_amd.ops import audit as A
from agent_hypervisor_amd.parallel.cp_merkle import (
    cp_merkle_root,
    local_block,
    merkle_root_of,
    simulated_cp_root,
)


def _leaves(n, seed=0):
    return A.hex_to_digests([hashlib.sha256(f"{seed}:{i}".encode()).hexdigest() for i in range(n)])


def _py_root(hexes):
    level = list(hexes)
    while len(level) > 1:
        if len(level) % 2:
            level.append(level[-1])
        level = [hashlib.sha256((level[i] + level[i + 1]).encode()).hexdigest() for i in range(0, len(level), 2)]
    return level[0]


@pytest.mark.parametrize("n", [1, 2, 3, 5, 7, 8, 9, 13, 31, 33, 100, 257])
@pytest.mark.parametrize("world", [1, 2, 3, 4, 8])
def test_simulated_cp_equals_serial(n, world):
    lv = _leaves(n, seed=n)
    want = _py_root(A.digests_to_hex(lv))
    assert A.digests_to_hex(merkle_root_of(lv))[0] == want
    assert A.digests_to_hex(simulated_cp_root(lv, world))[0] == want


def _worker(rank, world, port, n):
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        lv = _leaves(n, seed=42)
        s, e, _ = local_block(n, rank, world)
        root = cp_merkle_root(lv[s:e], n)
        assert A.digests_to_hex(root)[0] == _py_root(A.digests_to_hex(lv))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("n", [37, 4])
def test_cp_merkle_gloo_world3(n):
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    mp.start_processes(_worker, args=(3, port, n), nprocs=3, join=True, start_method="spawn")
