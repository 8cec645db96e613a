"""In-process "fake rank" world for the cross-rank merge math.

``run_ranks(world, fn)`` runs ``fn(rank)`` once per simulated rank, each on its
own thread, with a :class:`FakeGroup` installed as that thread's communicator for
``parallel.collectives``.  The group implements the subset of the
``torch.distributed`` surface the collectives use (``all_reduce`` with SUM / MIN /
MAX / PRODUCT, ``all_gather``, ``broadcast``, ``barrier``) over shared memory, and
reduces in rank order, so results are deterministic and independent of thread
scheduling.  It exercises the X01–X10 logic at any world size without process
spawn, rendezvous or sockets — the unit-test counterpart of the gloo (CPU) and
RCCL (MI355X) runs of the same functions.
"""

from __future__ import annotations

import threading
from typing import Any, Callable

import torch
import torch.distributed as dist


def _combine(a: torch.Tensor, b: torch.Tensor, op) -> torch.Tensor:
    if op == dist.ReduceOp.SUM:
        return a + b
    if op == dist.ReduceOp.MIN:
        return torch.minimum(a, b)
    if op == dist.ReduceOp.MAX:
        return torch.maximum(a, b)
    if op == dist.ReduceOp.PRODUCT:
        return a * b
    raise ValueError(f"fake group: unsupported reduce op {op}")


class FakeGroup:
    """A world of ``world`` threads sharing one rendezvous; ranks are thread-local."""

    def __init__(self, world: int) -> None:
        if world < 1:
            raise ValueError("world must be >= 1")
        self.world = world
        self._barrier = threading.Barrier(world)
        self._slots: list[Any] = [None] * world
        self._local = threading.local()

    # -- identity --------------------------------------------------------------
    def get_rank(self) -> int:
        return self._local.rank

    def get_world_size(self) -> int:
        return self.world

    # -- collectives -----------------------------------------------------------
    def _exchange(self, value: Any) -> list:
        self._slots[self.get_rank()] = value
        self._barrier.wait()
        vals = list(self._slots)
        self._barrier.wait()  # nobody overwrites a slot before everyone has read it
        return vals

    def all_reduce(self, tensor: torch.Tensor, op=dist.ReduceOp.SUM, async_op: bool = False):
        vals = self._exchange(tensor.clone())
        acc = vals[0]
        for v in vals[1:]:
            acc = _combine(acc, v, op)
        tensor.copy_(acc)
        return None

    def all_gather(self, out: list, tensor: torch.Tensor, async_op: bool = False):
        vals = self._exchange(tensor.clone())
        for o, v in zip(out, vals):
            o.copy_(v)
        return None

    def broadcast(self, tensor: torch.Tensor, src: int, async_op: bool = False):
        vals = self._exchange(tensor.clone())
        src_t = vals[src]
        if tensor.shape != src_t.shape:
            raise ValueError("fake group: broadcast shape mismatch")
        tensor.copy_(src_t)
        return None

    def barrier(self) -> None:
        self._barrier.wait()

    def abort(self) -> None:
        self._barrier.abort()


def run_ranks(world: int, fn: Callable[[int], Any]) -> list:
    """Run ``fn(rank)`` for every rank of a fresh :class:`FakeGroup`; return the
    per-rank results in rank order.  An exception on any rank aborts the
    rendezvous (so no rank waits forever) and is re-raised."""
    from agent_hypervisor_amd.parallel import collectives

    group = FakeGroup(world)
    results: list[Any] = [None] * world
    errors: list[BaseException | None] = [None] * world

    def body(rank: int) -> None:
        group._local.rank = rank
        collectives.set_thread_group(group)
        try:
            results[rank] = fn(rank)
        except threading.BrokenBarrierError as e:
            errors[rank] = e
        except BaseException as e:  # noqa: BLE001 - surfaced below
            errors[rank] = e
            group.abort()
        finally:
            collectives.set_thread_group(None)

    threads = [threading.Thread(target=body, args=(r,), name=f"fake-rank-{r}") for r in range(world)]
    for t in threads:
        t.start()
    for t in threads:
        t.join()
    first = next((e for e in errors if e is not None and not isinstance(e, threading.BrokenBarrierError)), None)
    if first is None:
        first = next((e for e in errors if e is not None), None)
    if first is not None:
        raise first
    return results
