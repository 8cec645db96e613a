"""Isolation levels: how much coordination a saga pays for.

Parity target: reference ``session/isolation.py:13-59``.  Declarative: the
properties tell a caller which machinery (vector clocks, intent locks) a level
needs; :func:`hypervisor.session.isolation.IsolationLevel.coordination_cost`
ranks them low / moderate / high.
"""

from __future__ import annotations

from enum import Enum

# level -> (vector clocks, intent locks, concurrent writes, cost)
_TRAITS = {
    "snapshot": (False, False, True, "low"),
    "read_committed": (True, False, True, "moderate"),
    "serializable": (True, True, False, "high"),
}


class IsolationLevel(str, Enum):
    SNAPSHOT = "snapshot"  # reads from a saga-start snapshot, buffered writes
    READ_COMMITTED = "read_committed"  # reads see the latest committed write
    SERIALIZABLE = "serializable"  # equivalent to some serial order

    @property
    def requires_vector_clocks(self) -> bool:
        return _TRAITS[self.value][0]

    @property
    def requires_intent_locks(self) -> bool:
        return _TRAITS[self.value][1]

    @property
    def allows_concurrent_writes(self) -> bool:
        return _TRAITS[self.value][2]

    @property
    def coordination_cost(self) -> str:
        return _TRAITS[self.value][3]
