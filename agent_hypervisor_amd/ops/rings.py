"""Ring kernels: K01 ring gate, K02 ring check (reference rings/enforcer.py,
models.py:34-42, 122-132)."""

from __future__ import annotations

from typing import Optional

import torch

from agent_hypervisor_amd.ops._launch import launch

# ActionFlag bits (csrc/include/ahv/semantics.h)
ACT_ADMIN = 1
ACT_READ_ONLY = 2
ACT_IRREVERSIBLE = 4


def action_flags(is_admin: bool, is_read_only: bool, irreversible: bool) -> int:
    return (ACT_ADMIN if is_admin else 0) | (ACT_READ_ONLY if is_read_only else 0) | (
        ACT_IRREVERSIBLE if irreversible else 0
    )


def ring_gate(sigma: torch.Tensor, consensus: Optional[torch.Tensor] = None) -> torch.Tensor:
    """ExecutionRing.from_sigma_eff for every element: fp64 σ → u8 ring (1/2/3)."""
    ring = torch.empty(sigma.shape, dtype=torch.uint8, device=sigma.device)
    launch(
        "ring_gate",
        {"n": sigma.numel()},
        {"sigma": sigma, "consensus": consensus, "ring": ring},
        {"sigma": torch.float64, "consensus": torch.uint8},
    )
    return ring


def ring_check(
    agent_ring: torch.Tensor,
    flags: torch.Tensor,
    sigma: torch.Tensor,
    consensus: torch.Tensor,
    witness: torch.Tensor,
) -> tuple[torch.Tensor, torch.Tensor]:
    """RingEnforcer.check for every element → (required ring, reason code).

    Reason codes are hypervisor.rings.enforcer.REASON_*; 0 = allowed."""
    n = agent_ring.numel()
    req = torch.empty(n, dtype=torch.uint8, device=agent_ring.device)
    reason = torch.empty(n, dtype=torch.uint8, device=agent_ring.device)
    u8 = torch.uint8
    launch(
        "ring_check",
        {"n": n},
        dict(agent_ring=agent_ring, action_flags=flags, sigma=sigma, consensus=consensus, witness=witness,
             required=req, reason=reason),
        dict(agent_ring=u8, action_flags=u8, sigma=torch.float64, consensus=u8, witness=u8),
    )
    return req, reason
