"""Agent-global liability on one rank's resident bond graph (X01/X02 partials).

:class:`ResidentBonds` keeps a rank's vouch edges device-resident in two CSR
views — by voucher (creation order within a row) for the K04 exposure partial,
and by vouchee for the K06 slash stage — sized for MI355X HBM (an edge costs
≈ 38 B: 4 M edges per 1 M agents ≈ 150 MB).  Kernels: ``agent_exposure`` and
``slash_clip`` in ``csrc/hip/global_liability.hip``; the cross-rank merges are
``collectives.allreduce_exposure`` (X01) and ``collectives.merge_slash_fixed``
(X02).
"""

from __future__ import annotations

import torch

from agent_hypervisor_amd.ops._launch import launch

f64, u8, i32, i64 = torch.float64, torch.uint8, torch.int32, torch.int64


class ResidentBonds:
    def __init__(self, n_agents: int, degree: int, device, seed: int = 0, max_bond: float = 0.2) -> None:
        dev = torch.device(device)
        A, E = int(n_agents), int(n_agents) * int(degree)
        g = torch.Generator(device=dev).manual_seed(seed)
        self.agents, self.edges, self.device = A, E, dev
        self.voucher = torch.arange(A, device=dev, dtype=i32).repeat_interleave(degree)
        self.vouchee = torch.randint(0, A, (E,), generator=g, device=dev, dtype=i32)
        self.bonded = torch.rand(E, generator=g, device=dev, dtype=f64) * max_bond
        self.offsets = torch.arange(0, E + 1, degree, device=dev, dtype=i64)
        self.active = torch.ones(E, device=dev, dtype=u8)
        self.expiry = torch.full((E,), -1, device=dev, dtype=i64)
        self.released = torch.zeros(E, device=dev, dtype=i64)
        order = torch.argsort(self.vouchee.to(i64), stable=True)
        self.in_edge = order.to(i32)
        self.in_src = self.voucher[order]
        counts = torch.bincount(self.vouchee.to(i64), minlength=A)
        self.in_offsets = torch.zeros(A + 1, device=dev, dtype=i64)
        self.in_offsets[1:] = torch.cumsum(counts, 0)

    @property
    def nbytes(self) -> int:
        ts = (self.voucher, self.vouchee, self.bonded, self.offsets, self.active, self.expiry, self.released,
              self.in_edge, self.in_src, self.in_offsets)
        return sum(t.numel() * t.element_size() for t in ts)

    def exposure(self, out: torch.Tensor, now_us: int = 0) -> torch.Tensor:
        """K04: out[a] = Σ live bonds agent a posted (creation-order fp64 sum per row)."""
        if out.dtype != f64 or out.numel() != self.agents:
            raise ValueError("out must be fp64 [agents]")
        launch("agent_exposure", {"agents": self.agents, "now_us": int(now_us)},
               {"offsets": self.offsets, "bonded": self.bonded, "active": self.active, "expiry": self.expiry,
                "out": out})
        return out

    def slash_clip(self, ids: torch.Tensor, omega: float, pair_id: torch.Tensor, pair_factor: torch.Tensor,
                   cursor: torch.Tensor, now_us: int = 0) -> None:
        """K06 stage: release every live bond posted for the slashed ``ids`` and emit
        (voucher, 1−ω) clip pairs into the fixed-capacity buffers (id −1 = unused)."""
        if pair_id.numel() != pair_factor.numel():
            raise ValueError("pair buffers differ in capacity")
        launch("slash_clip", {"k": int(ids.numel()), "cap": int(pair_id.numel()), "now_us": int(now_us),
                              "omega": float(omega)},
               {"ids": ids, "offsets": self.in_offsets, "src": self.in_src, "edge": self.in_edge,
                "active": self.active, "released": self.released, "expiry": self.expiry, "pair_id": pair_id,
                "pair_factor": pair_factor, "cursor": cursor},
               {"ids": i32, "pair_id": i32, "pair_factor": f64, "cursor": i64})
