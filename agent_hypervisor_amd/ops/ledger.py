"""Liability-ledger and verification kernels: K22 risk profiles and drift
severity, K21 fault-attribution raw scores (reference liability/ledger.py:103-169,
integrations/cmvk_adapter.py:240-250, liability/attribution.py:121-203)."""

from __future__ import annotations

import torch

from agent_hypervisor_amd.ops._launch import launch

u8, i32, f64 = torch.uint8, torch.int32, torch.float64

LEDGER_CODE = {
    "vouch_given": 0, "vouch_received": 1, "vouch_released": 2, "slash_received": 3, "slash_cascaded": 4,
    "quarantine_entered": 5, "quarantine_released": 6, "fault_attributed": 7, "clean_session": 8,
}
RECOMMENDATION = ("admit", "probation", "deny")
SEVERITY = ("none", "low", "medium", "high", "critical")


def risk_profiles(offsets: torch.Tensor, types: torch.Tensor, severity: torch.Tensor) -> dict:
    """Per-agent risk over agent-segmented ledger entries (entry order)."""
    A = offsets.numel() - 1
    dev = offsets.device
    out = dict(
        raw_risk=torch.empty(A, dtype=f64, device=dev),
        risk=torch.empty(A, dtype=f64, device=dev),
        recommendation=torch.empty(A, dtype=u8, device=dev),
        slash_count=torch.empty(A, dtype=i32, device=dev),
        quarantine_count=torch.empty(A, dtype=i32, device=dev),
        clean_count=torch.empty(A, dtype=i32, device=dev),
        fault_avg=torch.empty(A, dtype=f64, device=dev),
    )
    launch("ledger", {"agents": A}, dict(offsets=offsets, type=types, severity=severity, **out),
           dict(offsets=i32, type=u8, severity=f64))
    return out


def drift_severity(drift: torch.Tensor, low=0.15, medium=0.30, high=0.50, critical=0.75) -> torch.Tensor:
    sev = torch.empty(drift.numel(), dtype=u8, device=drift.device)
    launch("drift", {"n": drift.numel(), "low": low, "medium": medium, "high": high, "critical": critical},
           dict(drift=drift, severity=sev), dict(drift=f64))
    return sev


def attribution_raw(node_offsets, agent_offsets, agent_of_node, success, root_cause, risk_weight):
    """Raw per-agent contributions of each failure case (normalise on the host)."""
    G = int(agent_offsets[-1].item())
    dev = node_offsets.device
    raw = torch.zeros(G, dtype=f64, device=dev)
    cnt = torch.zeros(G, dtype=i32, device=dev)
    launch(
        "attribution",
        {"cases": node_offsets.numel() - 1},
        dict(node_offsets=node_offsets, agent_offsets=agent_offsets, agent_of_node=agent_of_node, success=success,
             root_cause=root_cause, risk_weight=risk_weight, raw=raw, node_count=cnt),
        dict(node_offsets=i32, agent_offsets=i32, agent_of_node=i32, success=u8, root_cause=u8, risk_weight=f64),
    )
    return raw
