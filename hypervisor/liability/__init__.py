"""Liability matrix: a standalone voucher→vouchee edge list for one session.

Parity target: reference ``liability/__init__.py:14-139``.  Independent of
:class:`~hypervisor.liability.vouching.VouchingEngine`.

* ``cascade_path(agent, max_depth=2)``: every voucher→vouchee path starting at
  ``agent`` explored depth-first, emitted at leaves and at every interior node
  with out-edges, limited to ``max_depth`` hops;
* ``has_cycle``: DFS with an on-stack set.
"""

from __future__ import annotations

from dataclasses import dataclass


@dataclass
class LiabilityEdge:
    voucher_did: str
    vouchee_did: str
    bonded_amount: float
    vouch_id: str


class LiabilityMatrix:
    def __init__(self, session_id: str) -> None:
        self.session_id = session_id
        self._edges: list[LiabilityEdge] = []

    def add_edge(self, voucher_did: str, vouchee_did: str, bonded_amount: float, vouch_id: str) -> LiabilityEdge:
        e = LiabilityEdge(voucher_did, vouchee_did, bonded_amount, vouch_id)
        self._edges.append(e)
        return e

    def remove_edge(self, vouch_id: str) -> None:
        self._edges = [e for e in self._edges if e.vouch_id != vouch_id]

    def who_vouches_for(self, agent_did: str) -> list[LiabilityEdge]:
        return [e for e in self._edges if e.vouchee_did == agent_did]

    def who_is_vouched_by(self, agent_did: str) -> list[LiabilityEdge]:
        return [e for e in self._edges if e.voucher_did == agent_did]

    def total_exposure(self, voucher_did: str) -> float:
        return sum(e.bonded_amount for e in self._edges if e.voucher_did == voucher_did)

    def cascade_path(self, agent_did: str, max_depth: int = 2) -> list[list[str]]:
        found: list[list[str]] = []

        def walk(node: str, trail: list[str]) -> None:
            if len(trail) > max_depth + 1:
                return
            outs = self.who_is_vouched_by(node)
            if not outs:
                if len(trail) > 1:
                    found.append(list(trail))
                return
            for e in outs:
                if e.vouchee_did in trail:
                    continue
                trail.append(e.vouchee_did)
                walk(e.vouchee_did, trail)
                trail.pop()
            if len(trail) > 1:
                found.append(list(trail))

        walk(agent_did, [agent_did])
        return found

    def has_cycle(self) -> bool:
        adj: dict[str, list[str]] = {}
        nodes: list[str] = []
        for e in self._edges:
            adj.setdefault(e.voucher_did, []).append(e.vouchee_did)
            nodes.extend((e.voucher_did, e.vouchee_did))
        WHITE, GREY, BLACK = 0, 1, 2
        color: dict[str, int] = {}

        def dfs(n: str) -> bool:
            color[n] = GREY
            for m in adj.get(n, ()):
                c = color.get(m, WHITE)
                if c == GREY:
                    return True
                if c == WHITE and dfs(m):
                    return True
            color[n] = BLACK
            return False

        return any(color.get(n, WHITE) == WHITE and dfs(n) for n in nodes)

    def clear(self) -> None:
        self._edges.clear()

    @property
    def edges(self) -> list[LiabilityEdge]:
        return list(self._edges)


__all__ = ["LiabilityEdge", "LiabilityMatrix"]
