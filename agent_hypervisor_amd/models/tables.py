"""Device-resident governance state: SoA tables owned by PyTorch.

Every engine row is a set of column tensors on the HIP device, addressed by dense
int32 ids from the interner.  Column names are the kernel argument names of
``csrc/include/ahv/pipeline.h`` (``SessionTables``), so a table passes itself to a
launcher as a dict of data pointers.

Sizing for MI355X (288 GB HBM3E per GPU): a session row is ~360 B with the
default 8-delta audit window, an agent row 20 B, a vouch edge 34 B — so one GPU
holds e.g. 10 M agents (0.2 GB) + 100 M vouch edges (3.4 GB) + 64 M live
sessions (23 GB) with most of HBM left for audit history.
"""

from __future__ import annotations

from dataclasses import dataclass

from typing import Optional

import torch

P_MAX = 16  # participant row width (kMaxParticipants)


def _z(shape, dtype, device):
    return torch.zeros(shape, dtype=dtype, device=device)


class SessionTable:
    """One row per session slot; slots are recycled ring-buffer style."""

    COLUMNS = (
        "sess_uuid", "sess_state", "sess_mode", "sess_creator", "sess_created_us", "sess_terminated_us",
        "part_count", "part_agent", "part_ring", "part_sigma_raw", "part_sigma_eff", "part_joined_us",
        "delta_hash", "delta_count", "merkle_root", "saga_uuid", "step_uuid", "saga_state", "step_state",
        "step_started_us", "step_completed_us", "committed_at_us", "gc_retained", "bonds_released", "status",
    )

    def __init__(self, capacity: int, device, dmax: int = 8) -> None:
        self.capacity = int(capacity)
        self.dmax = int(dmax)
        self.device = torch.device(device)
        c, d, dev = self.capacity, self.dmax, self.device
        self.sess_uuid = _z((c, 4), torch.int32, dev)
        self.sess_state = torch.full((c,), 255, dtype=torch.uint8, device=dev)
        self.sess_mode = _z((c,), torch.uint8, dev)
        self.sess_creator = _z((c,), torch.int32, dev)
        self.sess_created_us = _z((c,), torch.int64, dev)
        self.sess_terminated_us = _z((c,), torch.int64, dev)
        self.part_count = _z((c,), torch.int32, dev)
        self.part_agent = torch.full((c, P_MAX), -1, dtype=torch.int32, device=dev)
        self.part_ring = torch.full((c, P_MAX), 3, dtype=torch.uint8, device=dev)
        self.part_sigma_raw = _z((c, P_MAX), torch.float64, dev)
        self.part_sigma_eff = _z((c, P_MAX), torch.float64, dev)
        self.part_joined_us = _z((c, P_MAX), torch.int64, dev)
        self.delta_hash = _z((c, d, 8), torch.int32, dev)
        self.delta_count = _z((c,), torch.int32, dev)
        self.merkle_root = _z((c, 8), torch.int32, dev)
        self.saga_uuid = _z((c, 4), torch.int32, dev)
        self.step_uuid = _z((c, 4), torch.int32, dev)
        self.saga_state = _z((c,), torch.uint8, dev)
        self.step_state = _z((c,), torch.uint8, dev)
        self.step_started_us = _z((c,), torch.int64, dev)
        self.step_completed_us = _z((c,), torch.int64, dev)
        self.committed_at_us = _z((c,), torch.int64, dev)
        self.gc_retained = _z((c,), torch.int32, dev)
        self.bonds_released = _z((c,), torch.int32, dev)
        self.status = _z((c,), torch.int32, dev)

    def pointers(self) -> dict[str, int]:
        return {name: getattr(self, name).data_ptr() for name in self.COLUMNS}

    @property
    def nbytes(self) -> int:
        return sum(getattr(self, n).numel() * getattr(self, n).element_size() for n in self.COLUMNS)


class AgentTable:
    """Agent-global columns: σ_raw and the interned DID."""

    def __init__(self, capacity: int, device) -> None:
        self.capacity = int(capacity)
        self.device = torch.device(device)
        self.sigma = _z((self.capacity,), torch.float64, self.device)
        self.did = torch.full((self.capacity,), -1, dtype=torch.int32, device=self.device)
        self.count = 0

    def add(self, did_ids: torch.Tensor, sigmas: torch.Tensor) -> torch.Tensor:
        n = int(did_ids.numel())
        if self.count + n > self.capacity:
            raise RuntimeError(f"agent table full ({self.capacity} rows)")
        ids = torch.arange(self.count, self.count + n, dtype=torch.int32, device=self.device)
        self.did[self.count : self.count + n] = did_ids.to(self.device, torch.int32)
        self.sigma[self.count : self.count + n] = sigmas.to(self.device, torch.float64)
        self.count += n
        return ids


class VouchSlab:
    """Resident vouch edges of the pipeline's session slots: slot ``s`` owns
    edges ``[s·stride, s·stride + count[s])`` in creation order.  The pipeline
    kernel's terminate stage releases the active ones (K07, stamping
    ``released_us``) and empties the slot for the session that reuses it.
    Columns are allocated on the first :meth:`stage` (an engine that never
    vouches carries no slab)."""

    COLUMNS = ("voucher", "vouchee", "bonded", "active", "expiry_us", "released_us")

    def __init__(self, capacity: int, stride: int, device) -> None:
        self.capacity, self.stride, self.device = capacity, stride, torch.device(device)
        self.count: Optional[torch.Tensor] = None

    def _alloc(self) -> None:
        n, dev = self.capacity * self.stride, self.device
        self.count = _z((self.capacity,), torch.int32, dev)
        self.voucher = _z((n,), torch.int32, dev)
        self.vouchee = _z((n,), torch.int32, dev)
        self.bonded = _z((n,), torch.float64, dev)
        self.active = _z((n,), torch.uint8, dev)
        self.expiry_us = torch.full((n,), -1, dtype=torch.int64, device=dev)
        self.released_us = _z((n,), torch.int64, dev)

    @property
    def allocated(self) -> bool:
        return self.count is not None

    def stage(self, slots, voucher, vouchee, bonded, expiry_us=None) -> torch.Tensor:
        """Append edges (in the given order) to the slabs of ``slots``; returns
        their flat edge indices.  Raises if a slot would exceed ``stride``."""
        if not self.allocated:
            self._alloc()
        dev = self.device
        slots = torch.as_tensor(slots, dtype=torch.int64).to(dev)
        m = slots.numel()
        order = torch.sort(slots, stable=True).indices
        ss = slots[order]
        first = torch.ones(m, dtype=torch.bool, device=dev)
        if m > 1:
            first[1:] = ss[1:] != ss[:-1]
        start = torch.cummax(torch.where(first, torch.arange(m, device=dev), torch.zeros_like(ss)), 0).values
        rank = torch.empty(m, dtype=torch.int64, device=dev)
        rank[order] = torch.arange(m, device=dev) - start
        pos = self.count[slots].to(torch.int64) + rank
        if m and int(pos.max()) >= self.stride:
            raise ValueError(f"vouch slab holds {self.stride} edges per session slot")
        idx = slots * self.stride + pos
        self.voucher[idx] = torch.as_tensor(voucher, dtype=torch.int32).to(dev)
        self.vouchee[idx] = torch.as_tensor(vouchee, dtype=torch.int32).to(dev)
        self.bonded[idx] = torch.as_tensor(bonded, dtype=torch.float64).to(dev)
        self.active[idx] = 1
        self.expiry_us[idx] = -1 if expiry_us is None else torch.as_tensor(expiry_us, dtype=torch.int64).to(dev)
        self.released_us[idx] = 0
        self.count.index_add_(0, slots, torch.ones(m, dtype=torch.int32, device=dev))
        return idx
