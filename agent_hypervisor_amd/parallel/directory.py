"""Session directory: data-parallel session sharding.

Every session is owned by exactly one rank (one GPU).  All per-session state —
SSO, VFS, vouch edges, saga, delta chain — lives in that rank's device tables,
so the per-session governance path never communicates; only the agent-global
views of :mod:`agent_hypervisor_amd.parallel.collectives` do.

The directory is host metadata replicated on every rank: creation requests are
placed deterministically (round-robin, least-loaded or a stable hash of the
session id), so every rank computes the same owner without a round trip, and
saga ids route to their session's owner (X07: the reference scans every
session, server.py:418-505).
"""

from __future__ import annotations

import hashlib
from dataclasses import dataclass, field
from typing import Optional

POLICIES = ("round_robin", "least_loaded", "hash")


def stable_rank(key: str, world: int) -> int:
    """Process-independent owner of ``key`` (Python's hash() is salted)."""
    h = hashlib.blake2b(key.encode(), digest_size=8).digest()
    return int.from_bytes(h, "little") % world


@dataclass
class SessionDirectory:
    world: int = 1
    policy: str = "round_robin"
    _owner: dict[str, int] = field(default_factory=dict)
    _load: list[int] = field(default_factory=list)
    _sagas: dict[str, str] = field(default_factory=dict)
    _next: int = 0
    _dead: set = field(default_factory=set)

    def __post_init__(self) -> None:
        if self.world < 1:
            raise ValueError("world must be >= 1")
        if self.policy not in POLICIES:
            raise ValueError(f"unknown placement policy {self.policy!r}; valid: {POLICIES}")
        self._load = [0] * self.world

    # -- liveness ----------------------------------------------------------------
    def mark_dead(self, ranks) -> None:
        """Exclude failed ranks from placement and rebalancing (failover)."""
        self._dead.update(int(r) for r in ranks)
        if len(self._dead) >= self.world:
            raise RuntimeError("every rank is marked dead")

    def mark_alive(self, rank: int) -> None:
        self._dead.discard(int(rank))

    @property
    def live_ranks(self) -> list[int]:
        return [r for r in range(self.world) if r not in self._dead]

    # -- placement -------------------------------------------------------------
    def next_rank(self, key: Optional[str] = None) -> int:
        """The rank the next new session goes to (advances round-robin state).

        Used when the owner must mint the session id: place first, then
        :meth:`assign` the id the owner returned.  Dead ranks are skipped.
        """
        live = self.live_ranks
        if self.policy == "round_robin":
            for _ in range(self.world):
                r = self._next
                self._next = (self._next + 1) % self.world
                if r not in self._dead:
                    return r
            return live[0]
        if self.policy == "least_loaded":
            return min(live, key=lambda k: (self._load[k], k))
        r = stable_rank(key or str(len(self._owner)), self.world)
        return r if r not in self._dead else live[stable_rank(key or "", len(live))]

    def assign(self, session_id: str, rank: int) -> None:
        if session_id in self._owner:
            raise ValueError(f"session {session_id} already placed on rank {self._owner[session_id]}")
        self._owner[session_id] = rank
        self._load[rank] += 1

    def place(self, session_id: str) -> int:
        """Assign ``session_id`` to a rank (idempotent) and return it."""
        r = self._owner.get(session_id)
        if r is not None:
            return r
        r = self.next_rank(session_id)
        self._owner[session_id] = r
        self._load[r] += 1
        return r

    def owner(self, session_id: str) -> Optional[int]:
        return self._owner.get(session_id)

    def is_local(self, session_id: str, rank: int) -> bool:
        return self._owner.get(session_id) == rank

    def release(self, session_id: str) -> None:
        """Forget an archived session (its commitment stays with the audit log)."""
        r = self._owner.pop(session_id, None)
        if r is not None:
            self._load[r] -= 1
        for g in [g for g, s in self._sagas.items() if s == session_id]:
            del self._sagas[g]

    # -- saga routing (X07) -------------------------------------------------------
    def register_saga(self, saga_id: str, session_id: str) -> None:
        if session_id not in self._owner:
            raise KeyError(f"session {session_id} is not placed")
        self._sagas[saga_id] = session_id

    def route_saga(self, saga_id: str) -> Optional[tuple[int, str]]:
        s = self._sagas.get(saga_id)
        return (self._owner[s], s) if s is not None else None

    # -- views ------------------------------------------------------------------
    @property
    def load(self) -> list[int]:
        return list(self._load)

    def sessions_of(self, rank: int) -> list[str]:
        return [s for s, r in self._owner.items() if r == rank]

    def __len__(self) -> int:
        return len(self._owner)

    def rebalance_plan(self) -> list[tuple[str, int, int]]:
        """Moves (session, from, to) that level the per-rank load to within one
        session; executed with an all-to-all of the session rows (P08)."""
        live = self.live_ranks
        target = len(self._owner) // len(live)
        extra = len(self._owner) % len(live)
        want = [0] * self.world
        for i, k in enumerate(live):
            want[k] = target + (1 if i < extra else 0)
        load = list(self._load)
        donors = {k: [s for s, r in self._owner.items() if r == k] for k in range(self.world)}
        moves = []
        for dst in live:
            for src in range(self.world):
                while load[dst] < want[dst] and load[src] > want[src]:
                    s = donors[src].pop()
                    moves.append((s, src, dst))
                    load[src] -= 1
                    load[dst] += 1
        return moves

    def apply(self, moves: list[tuple[str, int, int]]) -> None:
        for s, src, dst in moves:
            if self._owner.get(s) != src:
                raise ValueError(f"session {s} is not owned by rank {src}")
            self._owner[s] = dst
            self._load[src] -= 1
            self._load[dst] += 1


def shard_counts(global_batch: int, world: int) -> list[int]:
    """Per-rank share of a global batch of new sessions (balanced to ±1)."""
    base, extra = divmod(global_batch, world)
    return [base + (1 if r < extra else 0) for r in range(world)]
