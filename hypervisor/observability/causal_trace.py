"""Causal trace ids: ``trace/span[/parent]`` identifiers of the spawn tree.

Parity target: reference ``observability/causal_trace.py:16-68``.  Frozen value
type; ``trace_id`` 12 hex, ``span_id`` 8 hex.  ``from_string`` needs ≥ 2 parts and
does not recover the depth (it becomes 0); ``is_ancestor_of`` compares trace id
and depth only (Q18, preserved).
"""

from __future__ import annotations

from dataclasses import dataclass, field
from typing import Optional

from agent_hypervisor_amd._native import C as _C


def _trace() -> str:
    return _C.hex_id("", 12)


def _span() -> str:
    return _C.hex_id("", 8)


@dataclass(frozen=True)
class CausalTraceId:
    trace_id: str = field(default_factory=_trace)
    span_id: str = field(default_factory=_span)
    parent_span_id: Optional[str] = None
    depth: int = 0

    def child(self) -> "CausalTraceId":
        return CausalTraceId(self.trace_id, _span(), self.span_id, self.depth + 1)

    def sibling(self) -> "CausalTraceId":
        return CausalTraceId(self.trace_id, _span(), self.parent_span_id, self.depth)

    @property
    def full_id(self) -> str:
        if self.parent_span_id:
            return f"{self.trace_id}/{self.span_id}/{self.parent_span_id}"
        return f"{self.trace_id}/{self.span_id}"

    @classmethod
    def from_string(cls, s: str) -> "CausalTraceId":
        parts = s.split("/")
        if len(parts) < 2:
            raise ValueError(f"Invalid causal trace ID: {s}")
        return cls(trace_id=parts[0], span_id=parts[1], parent_span_id=parts[2] if len(parts) > 2 else None)

    def is_ancestor_of(self, other: "CausalTraceId") -> bool:
        return self.trace_id == other.trace_id and other.depth > self.depth

    def __str__(self) -> str:
        return self.full_id
