"""Agent-sharded ownership of agent-global views (SURVEY P02 "TP analogue",
P03 stream overlap, P08 session re-sharding).

P02 — there are no weight matrices to split, but agent-global tables (global σ,
ledger risk, exposure by agent) have a natural owner: ``agent_id % world``
(here: contiguous ranges, so a reduce-scatter delivers each owner its slice).
:func:`reduce_to_owners` sums per-rank partial vectors and leaves every rank
with exactly the agents it owns — half the traffic of an all-reduce, and the
right shape for owner-routed queries (``GET /agents/{did}/liability`` asks the
owner only).

P03 — :class:`OverlappedCollective` issues a collective on a dedicated HIP
stream after an event recorded on the compute stream, so the next batch's
kernels overlap the exchange (epoch-cadence views never sit on the critical
path); ``wait()`` joins it back.

P08 — :func:`export_rows` / :func:`import_rows` move session-table rows between
engines; :func:`exchange_rows` ships them rank-to-rank with one all-to-all of
packed rows (rebalancing after failover or skewed placement).
"""

from __future__ import annotations

import math
from typing import Optional

import torch
import torch.distributed as dist

from agent_hypervisor_amd.models.engine import EngineSessions as SessionTable


def _world_rank() -> tuple[int, int]:
    if dist.is_available() and dist.is_initialized():
        return dist.get_world_size(), dist.get_rank()
    return 1, 0


def owned_range(n_agents: int, rank: int, world: int) -> tuple[int, int]:
    """[start, stop) of the agent ids owned by ``rank`` (balanced contiguous split)."""
    base, extra = divmod(n_agents, world)
    start = rank * base + min(rank, extra)
    return start, start + base + (1 if rank < extra else 0)


def owner_of(agent_id: int, n_agents: int, world: int) -> int:
    base, extra = divmod(n_agents, world)
    cut = extra * (base + 1)
    return agent_id // (base + 1) if agent_id < cut else extra + (agent_id - cut) // max(base, 1)


def reduce_to_owners(partial: torch.Tensor) -> torch.Tensor:
    """Sum per-rank partial agent vectors; return this rank's owned slice."""
    world, rank = _world_rank()
    n = partial.numel()
    s, e = owned_range(n, rank, world)
    if world == 1:
        return partial[s:e].clone()
    sizes = [owned_range(n, r, world) for r in range(world)]
    if all(b - a == sizes[0][1] - sizes[0][0] for a, b in sizes):
        out = torch.empty(e - s, dtype=partial.dtype, device=partial.device)
        try:
            dist.reduce_scatter_tensor(out, partial.contiguous())
            return out
        except (RuntimeError, NotImplementedError):
            pass  # backend without reduce-scatter (gloo): fall through
    full = partial.clone()
    dist.all_reduce(full)
    return full[s:e].clone()


class OverlappedCollective:
    """Run ``fn(tensor)`` (a collective) on a side stream overlapping compute."""

    def __init__(self, device: torch.device) -> None:
        self.device = torch.device(device)
        self.stream = torch.cuda.Stream(self.device) if self.device.type == "cuda" else None
        self._done = None

    def launch(self, fn, tensor: torch.Tensor) -> "OverlappedCollective":
        if self.stream is None:
            fn(tensor)
            return self
        ready = torch.cuda.Event()
        ready.record(torch.cuda.current_stream(self.device))
        self.stream.wait_event(ready)
        with torch.cuda.stream(self.stream):
            fn(tensor)
            tensor.record_stream(self.stream)
            self._done = torch.cuda.Event()
            self._done.record(self.stream)
        return self

    def wait(self) -> None:
        """Make the current stream wait for the collective (no host sync)."""
        if self._done is not None:
            torch.cuda.current_stream(self.device).wait_event(self._done)
            self._done = None


# ------------------------------------------------------------- P08 migration

def export_rows(engine, slots: torch.Tensor) -> dict[str, torch.Tensor]:
    """Copy the session-table rows ``slots`` out (all columns)."""
    idx = slots.to(engine.device, torch.int64)
    return {k: getattr(engine.sessions, k).index_select(0, idx) for k in SessionTable.COLUMNS}


def import_rows(engine, rows: dict[str, torch.Tensor], slots: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Write rows into ``slots`` (default: the next ring-buffer slots); returns the slots.

    Agent ids in participant columns refer to the *source* engine's agent table;
    engines that share a registration order (the bench and the sharded
    deployments register the same population) can move rows unchanged."""
    n = rows["sess_state"].shape[0]
    cap = engine.sessions.capacity
    if slots is None:
        slots = (torch.arange(n, device=engine.device) + engine._next_slot) % cap
        engine._next_slot = (engine._next_slot + n) % cap
    idx = slots.to(engine.device, torch.int64)
    for k in SessionTable.COLUMNS:
        getattr(engine.sessions, k).index_copy_(0, idx, rows[k].to(engine.device))
    return slots


def _pack(rows: dict[str, torch.Tensor]) -> tuple[torch.Tensor, list[tuple[str, torch.dtype, tuple]]]:
    """Rows → one uint8 matrix [n, row_bytes] (+ layout)."""
    n = rows["sess_state"].shape[0]
    parts, layout = [], []
    for k in SessionTable.COLUMNS:
        t = rows[k].detach().cpu().contiguous()
        shape = tuple(t.shape[1:])
        nb = math.prod(shape) * t.element_size()
        layout.append((k, t.dtype, shape))
        parts.append(t.reshape(n, -1).view(torch.uint8) if n else torch.zeros((0, nb), dtype=torch.uint8))
    return torch.cat(parts, dim=1), layout


def _unpack(buf: torch.Tensor, layout) -> dict[str, torch.Tensor]:
    out, off = {}, 0
    n = buf.shape[0]
    for k, dt, shape in layout:
        nb = math.prod(shape) * torch.empty(0, dtype=dt).element_size()
        out[k] = buf[:, off:off + nb].clone(memory_format=torch.contiguous_format).view(dt).reshape((n, *shape))
        off += nb
    return out


def exchange_rows(per_dest: list[dict[str, torch.Tensor]]) -> list[dict[str, torch.Tensor]]:
    """All-to-all of session rows: ``per_dest[r]`` goes to rank r; returns the
    rows received from every rank (index = source rank)."""
    world, rank = _world_rank()
    if len(per_dest) != world:
        raise ValueError("need one row set per rank")
    if world == 1:
        return [per_dest[0]]
    packed = [_pack(r) for r in per_dest]
    layout = packed[rank][1]
    row_bytes = packed[0][0].shape[1]
    # the collective runs where the backend lives (RCCL: device buffers; gloo: host)
    dev = torch.device("cuda", torch.cuda.current_device()) if dist.get_backend() == "nccl" else torch.device("cpu")
    counts = torch.tensor([p[0].shape[0] for p in packed], dtype=torch.int64, device=dev)
    recv_counts = torch.empty_like(counts)
    dist.all_to_all_single(recv_counts, counts)
    send = torch.cat([p[0] for p in packed]).to(dev)
    recv = torch.empty((int(recv_counts.sum()), row_bytes), dtype=torch.uint8, device=dev)
    dist.all_to_all_single(recv, send, output_split_sizes=recv_counts.tolist(), input_split_sizes=counts.tolist())
    recv, recv_counts = recv.cpu(), recv_counts.cpu()
    out, off = [], 0
    for c in recv_counts.tolist():
        out.append(_unpack(recv[off:off + c], layout))
        off += c
    return out
