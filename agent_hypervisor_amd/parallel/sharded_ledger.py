"""Liability ledger sharded by session owner, with X03 risk reduction.

Reference: ``liability/ledger.py:50-169`` (one process, one list of entries).
Sharded, each entry lives on the rank that owns its session (the
:class:`~agent_hypervisor_amd.parallel.sharded.ShardedHypervisor` directory, or
a stable hash for sessions it does not know), in that rank's ledger — the
device-resident :class:`hypervisor._device_engines.DeviceLiabilityLedger` when a
device is given (K22 scores the log in one launch).  A risk profile is additive
until the final clamp, so every rank computes its partials (raw risk, per-type
counts, fault severity sum, entry count) for the requested agents and one
collective step combines them:

* raw risk as int64 fixed point (2⁻⁴⁰) — an associative, order-independent sum
  (X03, :func:`agent_hypervisor_amd.parallel.collectives.allreduce_risk`);
* the counts and the fault sum as ordinary all-reduces.

The clamp to [0, 1], the 4-decimal rounding and the admit / probation / deny
thresholds are then applied exactly as ``LiabilityLedger.compute_risk_profile``.
All calls are SPMD: every rank calls the same method with the same arguments.
"""

from __future__ import annotations

from typing import Optional, Sequence

import torch
import torch.distributed as dist

from agent_hypervisor_amd.parallel.collectives import FIXED_POINT_SCALE
from agent_hypervisor_amd.parallel.directory import stable_rank
from hypervisor.liability.ledger import AgentRiskProfile, LedgerEntryType, LiabilityLedger

_KEYS = ("raw", "slash", "quarantine", "clean", "fault_sum", "fault_n", "total")
_SLASH = (LedgerEntryType.SLASH_RECEIVED, LedgerEntryType.SLASH_CASCADED)


def host_partials(ledger: LiabilityLedger, agent_dids: Sequence[str]) -> dict[str, torch.Tensor]:
    """The same partials from a host ledger (creation-order sums)."""
    from hypervisor.liability.ledger import risk_increment

    cols = {k: [] for k in _KEYS}
    for a in agent_dids:
        hist = ledger.get_agent_history(a)
        raw = fs = 0.0
        sl = qu = cl = fn = 0
        for e in hist:
            t = LedgerEntryType(e.entry_type)
            sl += t in _SLASH
            qu += t == LedgerEntryType.QUARANTINE_ENTERED
            cl += t == LedgerEntryType.CLEAN_SESSION
            if t == LedgerEntryType.FAULT_ATTRIBUTED:
                fs += e.severity
                fn += 1
            raw += risk_increment(t, e.severity)
        for k, v in zip(_KEYS, (raw, sl, qu, cl, fs, fn, len(hist))):
            cols[k].append(v)
    return {k: torch.tensor(v, dtype=torch.float64 if k in ("raw", "fault_sum") else torch.int64)
            for k, v in cols.items()}


class ShardedLedger:
    def __init__(self, shv=None, device: Optional[str] = None) -> None:
        self.shv = shv
        self.rank = dist.get_rank() if dist.is_initialized() else 0
        self.world = dist.get_world_size() if dist.is_initialized() else 1
        self.local = LiabilityLedger(device=device)
        self.device = device

    def owner(self, session_id: str) -> int:
        if self.shv is not None:
            return self.shv.owner(session_id)
        return stable_rank(session_id, self.world)

    def record(self, agent_did: str, entry_type, session_id: str = "", severity: float = 0.0, details: str = "",
               related_agent: Optional[str] = None):
        """Store the entry on its session's owner (every rank calls; one stores)."""
        if self.owner(session_id) == self.rank:
            return self.local.record(agent_did, entry_type, session_id, severity, details, related_agent)
        return None

    def _partials(self, agent_dids: Sequence[str]) -> dict[str, torch.Tensor]:
        if hasattr(self.local, "partials"):
            return self.local.partials(agent_dids)
        return host_partials(self.local, agent_dids)

    def compute_risk_profiles(self, agent_dids: Sequence[str]) -> list[AgentRiskProfile]:
        p = self._partials(agent_dids)
        group = getattr(self.shv, "data_group", None) if self.shv is not None else None
        if self.world > 1:
            dev = torch.device("cuda", torch.cuda.current_device()) if dist.get_backend() == "nccl" \
                else torch.device("cpu")
            fx = torch.round(p["raw"].to(dev) * FIXED_POINT_SCALE).to(torch.int64)  # X03
            ints = torch.stack([p[k].to(dev) for k in ("slash", "quarantine", "clean", "fault_n", "total")])
            fsum = p["fault_sum"].to(dev)
            for t in (fx, ints, fsum):
                dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)
            raw = fx.to(torch.float64) / FIXED_POINT_SCALE
            p = dict(raw=raw, fault_sum=fsum, **{k: ints[i] for i, k in enumerate(
                ("slash", "quarantine", "clean", "fault_n", "total"))})
        host = {k: v.cpu().tolist() for k, v in p.items()}
        out = []
        for i, a in enumerate(agent_dids):
            total = int(host["total"][i])
            if total == 0:
                out.append(AgentRiskProfile(agent_did=a, recommendation="admit"))
                continue
            risk = min(1.0, max(0.0, host["raw"][i]))
            fn = int(host["fault_n"][i])
            out.append(AgentRiskProfile(
                agent_did=a, total_entries=total, slash_count=int(host["slash"][i]),
                quarantine_count=int(host["quarantine"][i]), clean_session_count=int(host["clean"][i]),
                fault_score_avg=round(host["fault_sum"][i] / fn, 4) if fn else 0.0, risk_score=round(risk, 4),
                recommendation=self.local.recommendation_for(risk)))
        return out

    def compute_risk_profile(self, agent_did: str) -> AgentRiskProfile:
        return self.compute_risk_profiles([agent_did])[0]

    def should_admit(self, agent_did: str) -> tuple[bool, str]:
        prof = self.compute_risk_profile(agent_did)
        if prof.recommendation == "deny":
            return False, f"Risk score {prof.risk_score:.2f} exceeds threshold"
        return True, prof.recommendation
