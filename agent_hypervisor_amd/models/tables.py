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


@dataclass
class VouchTable:
    """Vouch edges in creation order (σ_eff sums must follow creation order)."""

    voucher: torch.Tensor
    vouchee: torch.Tensor
    session: torch.Tensor
    bonded: torch.Tensor
    pct: torch.Tensor
    active: torch.Tensor
    expiry_us: torch.Tensor
    released_us: torch.Tensor
    count: int = 0

    @classmethod
    def allocate(cls, capacity: int, device) -> "VouchTable":
        dev = torch.device(device)
        return cls(
            voucher=_z((capacity,), torch.int32, dev),
            vouchee=_z((capacity,), torch.int32, dev),
            session=_z((capacity,), torch.int32, dev),
            bonded=_z((capacity,), torch.float64, dev),
            pct=_z((capacity,), torch.float64, dev),
            active=_z((capacity,), torch.uint8, dev),
            expiry_us=torch.full((capacity,), -1, dtype=torch.int64, device=dev),
            released_us=_z((capacity,), torch.int64, dev),
        )
