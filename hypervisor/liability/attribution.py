"""Proportional fault attribution for a failed saga (Shapley-inspired).

Parity target: reference ``liability/attribution.py:17-207``.

For each agent, summed over that agent's action nodes:

* +0.5 (DIRECT) if the node is the root cause (its step and agent match the
  failure);
* +0.3 (ENABLING) / (# failed non-root nodes overall) for each failed non-root
  node;
* +0.2 (PROXIMITY) · ω(action, default 0.5) / (# nodes of that agent).

Raw scores are normalised to sum to 1 (a zero total divides by 1), both rounded
with ``round(x, 4)`` and sorted by descending liability.  ``dependencies`` are
recorded but not traversed (as in the reference).

The per-agent reduction is the segmented kernel K21; the final ``round`` stays on
the host because it is CPython's correctly-rounded decimal rounding.
"""

from __future__ import annotations

from dataclasses import dataclass, field
from datetime import datetime
from typing import Optional

from agent_hypervisor_amd._native import C as _C
from hypervisor._clock import now as _now


@dataclass
class CausalNode:
    node_id: str = field(default_factory=lambda: _C.hex_id("", 8))
    agent_did: str = ""
    action_id: str = ""
    step_id: str = ""
    timestamp: datetime = field(default_factory=_now)
    success: bool = True
    is_root_cause: bool = False
    dependencies: list[str] = field(default_factory=list)


@dataclass
class FaultAttribution:
    agent_did: str
    liability_score: float
    causal_contribution: float
    is_direct_cause: bool = False
    reason: str = ""


@dataclass
class AttributionResult:
    attribution_id: str = field(default_factory=lambda: _C.hex_id("attr:", 8))
    saga_id: str = ""
    session_id: str = ""
    timestamp: datetime = field(default_factory=_now)
    attributions: list[FaultAttribution] = field(default_factory=list)
    causal_chain_length: int = 0
    root_cause_agent: Optional[str] = None

    @property
    def agents_involved(self) -> list[str]:
        return [a.agent_did for a in self.attributions]

    def get_liability(self, agent_did: str) -> float:
        for a in self.attributions:
            if a.agent_did == agent_did:
                return a.liability_score
        return 0.0


_DIRECT, _CONTRIB = "Direct cause of failure", "Contributing factor"


def _fault(agent, share: float, contrib: float, direct: bool) -> FaultAttribution:
    f = object.__new__(FaultAttribution)
    f.__dict__.update(agent_did=agent, liability_score=share, causal_contribution=contrib, is_direct_cause=direct,
                      reason=_DIRECT if direct else _CONTRIB)
    return f


def _by_score(x: FaultAttribution) -> float:
    return x.liability_score


class CausalAttributor:
    DIRECT_CAUSE_WEIGHT = 0.5
    ENABLING_WEIGHT = 0.3
    PROXIMITY_WEIGHT = 0.2

    def __init__(self) -> None:
        self._history: list[AttributionResult] = []

    def build_causal_dag(
        self,
        agent_actions: dict[str, list[dict]],
        failure_step_id: str,
        failure_agent_did: str,
    ) -> list[CausalNode]:
        return [
            CausalNode(
                agent_did=agent,
                action_id=a.get("action_id", ""),
                step_id=a.get("step_id", ""),
                success=a.get("success", True),
                is_root_cause=(a.get("step_id") == failure_step_id and agent == failure_agent_did),
                dependencies=a.get("dependencies", []),
            )
            for agent, acts in agent_actions.items()
            for a in acts
        ]

    def raw_scores(
        self, nodes: list[CausalNode], agents, risk_weights: dict[str, float]
    ) -> dict[str, float]:
        enabling_n = max(1, sum(1 for n in nodes if not n.success and not n.is_root_cause))
        per_agent: dict[str, list[CausalNode]] = {}
        for n in nodes:
            per_agent.setdefault(n.agent_did, []).append(n)
        out: dict[str, float] = {}
        for agent in agents:
            mine = per_agent.get(agent, [])
            denom = max(1, len(mine))
            s = 0.0
            for n in mine:
                if n.is_root_cause:
                    s += self.DIRECT_CAUSE_WEIGHT
                if not n.success and not n.is_root_cause:
                    s += self.ENABLING_WEIGHT / enabling_n
                s += self.PROXIMITY_WEIGHT * risk_weights.get(n.action_id, 0.5) / denom
            out[agent] = s
        return out

    def attribute(
        self,
        saga_id: str,
        session_id: str,
        agent_actions: dict[str, list[dict]],
        failure_step_id: str,
        failure_agent_did: str,
        risk_weights: Optional[dict[str, float]] = None,
    ) -> AttributionResult:
        nodes = self.build_causal_dag(agent_actions, failure_step_id, failure_agent_did)
        raw = self.raw_scores(nodes, set(agent_actions.keys()), risk_weights or {})
        return self._result(saga_id, session_id, nodes, raw, failure_agent_did)

    def _result(self, saga_id, session_id, nodes, raw: dict[str, float], failure_agent_did) -> AttributionResult:
        total = sum(raw.values()) or 1.0
        attrs = [
            FaultAttribution(
                agent_did=a,
                liability_score=round(r / total, 4),
                causal_contribution=round(r, 4),
                is_direct_cause=a == failure_agent_did,
                reason="Direct cause of failure" if a == failure_agent_did else "Contributing factor",
            )
            for a, r in raw.items()
        ]
        attrs.sort(key=lambda x: x.liability_score, reverse=True)
        res = AttributionResult(
            saga_id=saga_id,
            session_id=session_id,
            attributions=attrs,
            causal_chain_length=len(nodes),
            root_cause_agent=failure_agent_did,
        )
        self._history.append(res)
        return res

    def attribute_batch(self, cases, device="cpu") -> list[AttributionResult]:
        """:meth:`attribute` for many failure cases — dicts of its keyword
        arguments — with the raw per-agent scores of all cases from one K21
        launch on ``device``.  The cases' dicts are read into the kernel's columns
        natively (``_C.pack_attribution``; no :class:`CausalNode` objects — a
        result records only the chain length), the scores are rounded natively
        with CPython ``round``'s exact result (``_C.round_many``), and agents are
        ranked from the same set order as :meth:`attribute`, so ties sort
        identically."""
        import numpy as np
        import torch

        from agent_hypervisor_amd.ops import ledger as LG

        cases = cases if isinstance(cases, list) else list(cases)
        no, ao, aof, sc, rc, om, agents_of = _C.pack_attribution(cases)  # columns read natively
        node_off = np.frombuffer(no, dtype=np.int32)
        agent_off = np.frombuffer(ao, dtype=np.int32)
        C, N = len(cases), len(aof) // 4
        ints = torch.from_numpy(np.concatenate([node_off, agent_off, np.frombuffer(aof, dtype=np.int32)])).to(device)
        flags = torch.from_numpy(np.concatenate([np.frombuffer(sc, dtype=np.uint8),
                                                 np.frombuffer(rc, dtype=np.uint8)]).reshape(2, N)).to(device)
        raw = LG.attribution_raw(ints[: C + 1], ints[C + 1: 2 * C + 2], ints[2 * C + 2:], flags[0].contiguous(),
                                 flags[1].contiguous(), torch.from_numpy(np.frombuffer(om, dtype=np.float64).copy())
                                 .to(device))
        raw = raw.cpu().tolist()
        # normalisation in case order, CPython rounding done natively for all cases at once
        off = agent_off.tolist()
        totals = [sum(raw[off[k]: off[k + 1]]) or 1.0 for k in range(C)]
        share = C and _C.round_many([r / totals[k] for k in range(C) for r in raw[off[k]: off[k + 1]]], 4)
        contrib = C and _C.round_many(raw, 4)
        nodes = (node_off[1:] - node_off[:-1]).tolist()
        out = []
        for k, c in enumerate(cases):
            fa = c["failure_agent_did"]
            lo, hi = off[k], off[k + 1]
            attrs = [_fault(a, share[q], contrib[q], a == fa) for a, q in zip(agents_of[k], range(lo, hi))]
            attrs.sort(key=_by_score, reverse=True)
            res = AttributionResult(saga_id=c["saga_id"], session_id=c["session_id"], attributions=attrs,
                                    causal_chain_length=nodes[k], root_cause_agent=fa)
            self._history.append(res)
            out.append(res)
        return out

    def attribute_tensors(self, node_offsets, agent_offsets, agent_of_node, success, root_cause, risk_weight):
        """Tensor-native K21 (inputs on one device, int32 CSR offsets per case /
        agent, u8 flags, fp64 ω per node) → (raw, normalised) fp64 scores per
        (case, agent) on that device; a zero case total divides by 1."""
        import torch

        from agent_hypervisor_amd.ops import ledger as LG

        raw = LG.attribution_raw(node_offsets, agent_offsets, agent_of_node, success, root_cause, risk_weight)
        counts = (agent_offsets[1:] - agent_offsets[:-1]).to(torch.int64)
        case = torch.repeat_interleave(torch.arange(counts.numel(), device=raw.device), counts)
        total = torch.zeros(counts.numel(), dtype=raw.dtype, device=raw.device).index_add_(0, case, raw)
        total = torch.where(total == 0, torch.ones_like(total), total)
        return raw, raw / total[case]

    def _result_n(self, saga_id, session_id, n_nodes: int, agents, vals, failure_agent_did) -> AttributionResult:
        total = sum(vals) or 1.0
        attrs = [
            FaultAttribution(
                agent_did=a,
                liability_score=round(r / total, 4),
                causal_contribution=round(r, 4),
                is_direct_cause=a == failure_agent_did,
                reason="Direct cause of failure" if a == failure_agent_did else "Contributing factor",
            )
            for a, r in zip(agents, vals)
        ]
        attrs.sort(key=lambda x: x.liability_score, reverse=True)
        res = AttributionResult(saga_id=saga_id, session_id=session_id, attributions=attrs,
                                causal_chain_length=n_nodes, root_cause_agent=failure_agent_did)
        self._history.append(res)
        return res

    @property
    def attribution_history(self) -> list[AttributionResult]:
        return list(self._history)
