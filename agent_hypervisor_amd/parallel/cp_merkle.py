"""Context-parallel Merkle roots of very long audit chains.

The reference's Merkle tree (delta.py:117-134) pairs nodes level by level and
duplicates the last node of an odd level.  Split the leaf range into aligned
blocks of B = 2^k leaves, one block per rank:

* inside a block every level starts at an even global index, so the block's
  own tree is exactly the global tree restricted to it;
* the last (partial) block's root at its natural height h must be lifted to
  height k by self-pairing ``node(r, r)`` k − h times — at each of those levels
  it is the last, unpaired node of the global level;
* the W block roots are then the global tree's level-k nodes, and the
  ordinary Merkle over them (with odd duplication) is the global root.

So each rank reduces its contiguous leaf range locally (device kernel K09), and
one ``all_gather`` of 32-byte subtree roots (X10) lets every rank finish the
top levels.  The delta *chain* hash stays serial; only the tree parallelises.
"""

from __future__ import annotations

import math

import torch
import torch.distributed as dist

from agent_hypervisor_amd.ops import audit as A


def block_height(n_leaves: int, world: int) -> int:
    """k such that 2^k-leaf blocks cover ``n_leaves`` with at most ``world`` blocks."""
    per = max(1, math.ceil(n_leaves / world))
    return max(0, math.ceil(math.log2(per)))


def _node(x: torch.Tensor) -> torch.Tensor:
    """node(x, x) for a [1, 8] digest."""
    two = torch.cat([x, x]).contiguous()
    return A.merkle_roots(torch.tensor([0, 2], dtype=torch.int32, device=x.device), two)


def subtree_root(leaves: torch.Tensor, height: int) -> torch.Tensor:
    """Root of ``leaves`` ([n, 8] int32 digests, n ≤ 2^height) lifted to ``height``."""
    n = leaves.shape[0]
    if n == 0:
        raise ValueError("empty block")
    if n > (1 << height):
        raise ValueError(f"{n} leaves exceed a height-{height} block")
    r = A.merkle_tree_root(leaves.contiguous()).reshape(1, 8)  # K09 work-parallel (LDS subtrees, multi-pass)
    for _ in range(height - (math.ceil(math.log2(n)) if n > 1 else 0)):
        r = _node(r)
    return r


def top_root(block_roots: torch.Tensor) -> torch.Tensor:
    n = block_roots.shape[0]
    return A.merkle_roots(torch.tensor([0, n], dtype=torch.int32, device=block_roots.device),
                          block_roots.contiguous())


def local_block(n_leaves: int, rank: int, world: int) -> tuple[int, int, int]:
    """(start, stop, height) of the leaf range rank ``rank`` reduces."""
    k = block_height(n_leaves, world)
    b = 1 << k
    start = min(n_leaves, rank * b)
    return start, min(n_leaves, start + b), k


def cp_merkle_root(local_leaves: torch.Tensor, n_leaves: int, group=None) -> torch.Tensor:
    """Global Merkle root from each rank's block (``local_block`` ranges).

    Every rank passes the digests of its own range (possibly empty) and gets
    the global root back ([1, 8] int32)."""
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    rank = dist.get_rank(group) if dist.is_initialized() else 0
    start, stop, k = local_block(n_leaves, rank, world)
    if local_leaves.shape[0] != stop - start:
        raise ValueError(f"rank {rank} must hold leaves [{start}, {stop})")
    dev = local_leaves.device
    mine = subtree_root(local_leaves, k) if stop > start else torch.zeros((1, 8), dtype=torch.int32, device=dev)
    if world == 1:
        return mine
    gathered = [torch.empty_like(mine) for _ in range(world)]
    dist.all_gather(gathered, mine, group=group)
    nblocks = math.ceil(n_leaves / (1 << k))
    return top_root(torch.cat(gathered[:nblocks]))


def simulated_cp_root(leaves: torch.Tensor, world: int) -> torch.Tensor:
    """Single-process evaluation of the CP decomposition (tests, planning)."""
    n = leaves.shape[0]
    roots = []
    for r in range(world):
        s, e, k = local_block(n, r, world)
        if e > s:
            roots.append(subtree_root(leaves[s:e], k))
    return top_root(torch.cat(roots))


def merkle_root_of(leaves: torch.Tensor) -> torch.Tensor:
    n = leaves.shape[0]
    return A.merkle_roots(torch.tensor([0, n], dtype=torch.int32, device=leaves.device), leaves.contiguous())


__all__ = ["block_height", "local_block", "subtree_root", "top_root", "cp_merkle_root", "simulated_cp_root",
           "merkle_root_of"]
