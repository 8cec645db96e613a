"""Direct RCCL communicator (N06) for collectives enqueued on engine streams.

``torch.distributed`` with backend ``"nccl"`` is RCCL as well and remains the
default for the governance views (:mod:`.collectives`).  :class:`Communicator`
wraps a C++-owned ``ncclComm_t`` instead, so a collective can be issued on any
HIP stream — including inside a captured hipGraph — with no ProcessGroup in
the loop.  Bootstrapping only needs some torch.distributed group (``gloo`` is
enough) to broadcast the 128-byte unique id.

xGMI sizing note: MI355X links are point-to-point (7 × ≈153 GB/s per GPU), so
ring all-reduce is bound per link; the governance views are small (≤ tens of MB
per epoch) and latency-bound, which is why they are batched per epoch rather
than per session.
"""

from __future__ import annotations

from typing import Optional

import torch
import torch.distributed as dist

from agent_hypervisor_amd._native import C

_DT = {
    torch.int8: "int8", torch.uint8: "uint8", torch.int32: "int32", torch.int64: "int64",
    torch.float16: "float16", torch.bfloat16: "bfloat16", torch.float32: "float32", torch.float64: "float64",
}


def _dtype(t: torch.Tensor) -> str:
    try:
        return _DT[t.dtype]
    except KeyError:
        raise TypeError(f"RCCL does not support {t.dtype}") from None


def _stream(t: torch.Tensor, stream: Optional[torch.cuda.Stream]) -> int:
    return (stream or torch.cuda.current_stream(t.device)).cuda_stream


def _check(t: torch.Tensor) -> None:
    if t.device.type != "cuda":
        raise ValueError("RCCL collectives need device tensors")
    if not t.is_contiguous():
        raise ValueError("RCCL collectives need contiguous tensors")


class Communicator:
    """One RCCL communicator per process (one process per GPU)."""

    def __init__(self, rank: int, world: int, unique_id: bytes, device: int) -> None:
        self._c = C.RcclComm(rank, world, unique_id, device)
        self.rank, self.world, self.device = rank, world, device

    @classmethod
    def from_process_group(cls, device: Optional[int] = None, group=None) -> "Communicator":
        """Create on every rank of ``group`` (default: the world group)."""
        if dist.is_initialized():
            rank, world = dist.get_rank(group), dist.get_world_size(group)
        else:
            rank, world = 0, 1
        dev = torch.cuda.current_device() if device is None else device
        # RCCL's bootstrap queries the current HIP device: make sure torch has
        # created its context on it first (torch initialises HIP lazily).
        torch.cuda.set_device(dev)
        torch.empty(1, device=torch.device("cuda", dev)).zero_()
        torch.cuda.synchronize(dev)
        uid = [C.rccl_unique_id() if rank == 0 else None]
        if world > 1:
            dist.broadcast_object_list(uid, src=0, group=group)
        return cls(rank, world, uid[0], dev)

    @staticmethod
    def version() -> int:
        return C.rccl_version()

    # -- collectives (in place unless an output is given) --------------------------
    def all_reduce(self, t: torch.Tensor, op: str = "sum", stream=None) -> torch.Tensor:
        _check(t)
        self._c.all_reduce(t.data_ptr(), t.data_ptr(), t.numel(), _dtype(t), op, _stream(t, stream))
        return t

    def all_gather(self, t: torch.Tensor, out: Optional[torch.Tensor] = None, stream=None) -> torch.Tensor:
        _check(t)
        out = out if out is not None else torch.empty((self.world, *t.shape), dtype=t.dtype, device=t.device)
        _check(out)
        if out.numel() != t.numel() * self.world:
            raise ValueError("all_gather output must hold world × input elements")
        self._c.all_gather(t.data_ptr(), out.data_ptr(), t.numel(), _dtype(t), _stream(t, stream))
        return out

    def reduce_scatter(self, t: torch.Tensor, op: str = "sum", stream=None) -> torch.Tensor:
        _check(t)
        if t.numel() % self.world:
            raise ValueError("reduce_scatter input must split evenly across ranks")
        out = torch.empty(t.numel() // self.world, dtype=t.dtype, device=t.device)
        self._c.reduce_scatter(t.data_ptr(), out.data_ptr(), out.numel(), _dtype(t), op, _stream(t, stream))
        return out

    def broadcast(self, t: torch.Tensor, root: int = 0, stream=None) -> torch.Tensor:
        _check(t)
        self._c.broadcast(t.data_ptr(), t.data_ptr(), t.numel(), _dtype(t), root, _stream(t, stream))
        return t

    def all_to_all(self, t: torch.Tensor, stream=None) -> torch.Tensor:
        """Equal-block exchange: row block r of ``t`` goes to rank r (P08 re-shard)."""
        _check(t)
        if t.numel() % self.world:
            raise ValueError("all_to_all input must split evenly across ranks")
        out = torch.empty_like(t)
        self._c.all_to_all(t.data_ptr(), out.data_ptr(), t.numel() // self.world, _dtype(t), t.element_size(),
                           _stream(t, stream))
        return out

    def destroy(self) -> None:
        self._c.destroy()

    def async_error(self) -> str:
        """RCCL's asynchronous error text ("" while healthy)."""
        return self._c.async_error()

    def abort(self) -> None:
        """Abort (not wait for) pending collectives — used by the watchdog when a peer is lost."""
        self._c.abort()
