"""Vector clocks for causal consistency of session writes.

Parity target: reference ``session/vector_clock.py:19-165``.

* A :class:`VectorClock` is a sparse ``agent → counter`` map; absent agents read
  as 0, both for comparisons and for equality.
* ``happens_before(a, b)``: every component ``a ≤ b`` and at least one ``<``.
* ``VectorClockManager.write(strict=True)`` rejects a write only when the agent's
  clock strictly happens-before the path clock (it has not read the latest
  version); equal or concurrent clocks are admitted.  On success the agent
  ticks and the path clock becomes ``merge(path, agent)``.

The batched gfx950 path (kernel K19 in ``csrc/hip/session_kernels.hip``) stores
dense ``[paths, agents]`` u32 clocks for sessions with ≤ 64 agents and applies the
identical rule; see ``agent_hypervisor_amd.ops.session_ops``.
"""

from __future__ import annotations

from hypervisor._devsel import device_variant

from dataclasses import dataclass, field


class CausalViolationError(Exception):
    """A write from an agent whose view of the path is stale."""


@dataclass
class VectorClock:
    clocks: dict[str, int] = field(default_factory=dict)

    def tick(self, agent_did: str) -> None:
        self.clocks[agent_did] = self.clocks.get(agent_did, 0) + 1

    def get(self, agent_did: str) -> int:
        return self.clocks.get(agent_did, 0)

    def merge(self, other: "VectorClock") -> "VectorClock":
        out = dict(self.clocks)
        for a, c in other.clocks.items():
            out[a] = max(out.get(a, 0), c)
        return VectorClock(clocks=out)

    def _compare(self, other: "VectorClock") -> tuple[bool, bool]:
        """(all self ≤ other, any self < other) over the union of agents."""
        mine, theirs = self.clocks, other.clocks
        le, lt = True, False
        for a in mine.keys() | theirs.keys():
            x, y = mine.get(a, 0), theirs.get(a, 0)
            if x > y:
                le = False
                break
            if x < y:
                lt = True
        return le, lt

    def happens_before(self, other: "VectorClock") -> bool:
        le, lt = self._compare(other)
        return le and lt

    def is_concurrent(self, other: "VectorClock") -> bool:
        return not self.happens_before(other) and not other.happens_before(self)

    def copy(self) -> "VectorClock":
        return VectorClock(clocks=dict(self.clocks))

    def __eq__(self, other: object) -> bool:
        if not isinstance(other, VectorClock):
            return False
        mine, theirs = self.clocks, other.clocks
        return all(mine.get(a, 0) == theirs.get(a, 0) for a in mine.keys() | theirs.keys())

    __hash__ = None  # mutable, compared by value


class VectorClockManager:
    """Per-path and per-agent clocks for one session's shared state."""

    def __new__(cls, *args, device=None, **kwargs):
        """``device=...`` → the device-resident DeviceVectorClockManager (batched kernel path)."""
        return device_variant(cls, VectorClockManager, "DeviceVectorClockManager", device)

    def __init__(self, device=None) -> None:
        self._path_clocks: dict[str, VectorClock] = {}
        self._agent_clocks: dict[str, VectorClock] = {}
        self._conflict_count: int = 0

    def read(self, path: str, agent_did: str) -> VectorClock:
        pc = self._path_clocks.get(path) or VectorClock()
        ac = self._agent_clocks.get(agent_did) or VectorClock()
        self._agent_clocks[agent_did] = ac.merge(pc)
        return pc.copy()

    def write(self, path: str, agent_did: str, strict: bool = True) -> VectorClock:
        pc = self._path_clocks.get(path) or VectorClock()
        ac = self._agent_clocks.get(agent_did) or VectorClock()
        if strict and pc.clocks and ac.happens_before(pc):
            self._conflict_count += 1
            raise CausalViolationError(
                f"Agent {agent_did} has stale state for {path}. "
                f"Agent clock: {ac.clocks}, Path clock: {pc.clocks}. "
                "Must re-read before writing."
            )
        ac.tick(agent_did)
        merged = pc.merge(ac)
        self._path_clocks[path] = merged
        self._agent_clocks[agent_did] = ac
        return merged

    def apply_batch(self, ops, strict: bool = True) -> list[bool]:
        """``("read"|"write", path, agent_did)`` operations in order → ok flags
        (False: the write was rejected as causally stale and counted)."""
        out = []
        for op, path, agent in ops:
            if op == "write":
                try:
                    self.write(path, agent, strict)
                except CausalViolationError:
                    out.append(False)
                    continue
            else:
                self.read(path, agent)
            out.append(True)
        return out

    def get_path_clock(self, path: str) -> VectorClock:
        c = self._path_clocks.get(path)
        return c.copy() if c is not None else VectorClock()

    def get_agent_clock(self, agent_did: str) -> VectorClock:
        c = self._agent_clocks.get(agent_did)
        return c.copy() if c is not None else VectorClock()

    @property
    def conflict_count(self) -> int:
        return self._conflict_count

    @property
    def tracked_paths(self) -> int:
        return len(self._path_clocks)
