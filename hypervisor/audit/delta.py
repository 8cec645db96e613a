"""Delta audit engine: Merkle-chained semantic deltas of VFS state.

Parity target: reference ``audit/delta.py:17-160`` — this is the on-wire audit
format and it is byte-exact:

* ``SemanticDelta.compute_hash`` = SHA-256 of ``json.dumps(payload,
  sort_keys=True)`` over ``delta_id, turn_id, session_id, agent_did,
  timestamp.isoformat(), changes[{path, operation, content_hash,
  previous_hash}], parent_hash`` (``VFSChange.agent_did`` is not hashed);
* ``capture`` increments the turn, links ``parent_hash`` to the previous delta,
  defaults ``delta_id`` to ``delta:{turn}`` and hashes immediately;
* the Merkle root hashes the ASCII of ``hex(left) + hex(right)`` level by level,
  duplicating the last node of odd levels; a single delta is its own root.

The canonical payload is rendered and hashed by the native core
(``agent_hypervisor_amd._C.delta_hash``; shared SHA-256 with the gfx950 batched
audit kernels K08/K09/K10).  Exotic field types that ``json.dumps`` would render
differently from the fast path (non-str ids, bool turn ids …) are hashed through
``json.dumps`` itself, so the digest is always the reference's.

Fix: :meth:`DeltaEngine.verify_chain` recomputes hashes
without writing them back, so tampering with the last delta or with a stored
hash is detected.  Parity mode restores the reference's self-"repairing" verify.
"""

from __future__ import annotations

import hashlib
import json
from dataclasses import dataclass
from datetime import datetime
from typing import Optional

from agent_hypervisor_amd._native import C as _C
from hypervisor import config as _cfg
from hypervisor._clock import now as _now

_native_delta_hash = _C.delta_hash
_native_payload = _C.delta_payload
_native_merkle = _C.merkle_root


@dataclass
class VFSChange:
    path: str
    operation: str  # add | modify | delete | permission
    content_hash: Optional[str] = None
    previous_hash: Optional[str] = None
    agent_did: Optional[str] = None


def _payload_json(d: "SemanticDelta") -> str:
    return json.dumps(
        {
            "delta_id": d.delta_id,
            "turn_id": d.turn_id,
            "session_id": d.session_id,
            "agent_did": d.agent_did,
            "timestamp": d.timestamp.isoformat(),
            "changes": [
                {
                    "path": c.path,
                    "operation": c.operation,
                    "content_hash": c.content_hash,
                    "previous_hash": c.previous_hash,
                }
                for c in d.changes
            ],
            "parent_hash": d.parent_hash,
        },
        sort_keys=True,
    )


def canonical_payload(d: "SemanticDelta") -> bytes:
    """The exact bytes that are hashed for ``d`` (the self-verifying log record)."""
    b = _native_payload(d)
    return b if b is not None else _payload_json(d).encode()


def delta_digest(d: "SemanticDelta") -> str:
    """Hex digest of ``d``'s canonical payload, without mutating ``d``."""
    h = _native_delta_hash(d)
    if h is None:
        h = hashlib.sha256(_payload_json(d).encode()).hexdigest()
    return h


@dataclass
class SemanticDelta:
    delta_id: str
    turn_id: int
    session_id: str
    agent_did: str
    timestamp: datetime
    changes: list[VFSChange]
    parent_hash: Optional[str]
    delta_hash: str = ""

    def compute_hash(self) -> str:
        self.delta_hash = delta_digest(self)
        return self.delta_hash


class DeltaEngine:
    def __init__(self, session_id: str) -> None:
        self.session_id = session_id
        self._deltas: list[SemanticDelta] = []
        self._turn_counter = 0

    def capture(
        self,
        agent_did: str,
        changes: list[VFSChange],
        delta_id: Optional[str] = None,
    ) -> SemanticDelta:
        self._turn_counter = turn = self._turn_counter + 1
        ds = self._deltas
        d = SemanticDelta(
            delta_id or f"delta:{turn}",
            turn,
            self.session_id,
            agent_did,
            _now(),
            changes,
            ds[-1].delta_hash if ds else None,
        )
        h = _native_delta_hash(d)
        d.delta_hash = h if h is not None else hashlib.sha256(_payload_json(d).encode()).hexdigest()
        ds.append(d)
        return d

    def compute_merkle_root(self) -> Optional[str]:
        if not self._deltas:
            return None
        return _native_merkle([d.delta_hash for d in self._deltas])

    def verify_chain(self) -> bool:
        mutate = _cfg.parity_mode()
        prev: Optional[str] = None
        for i, d in enumerate(self._deltas):
            expected = d.compute_hash() if mutate else delta_digest(d)
            if d.delta_hash != expected:
                return False
            if i == 0:
                if d.parent_hash is not None:
                    return False
            elif d.parent_hash != prev:
                return False
            prev = d.delta_hash
        return True

    @property
    def deltas(self) -> list[SemanticDelta]:
        return list(self._deltas)

    @property
    def turn_count(self) -> int:
        return self._turn_counter

    # -- on-disk audit log ------------------------------------
    def export_records(self) -> list[dict]:
        """Self-verifying records: canonical payload text + stored digest."""
        return [
            {"payload": canonical_payload(d).decode("ascii"), "delta_hash": d.delta_hash}
            for d in self._deltas
        ]

    def prune_expired(self, retention_days: int) -> int:
        """Drop deltas older than the retention window (GC hook); returns count.

        The Merkle root of a pruned engine no longer covers the dropped deltas,
        so the GC only calls this after the root has been committed.
        """
        from datetime import timedelta

        cutoff = _now() - timedelta(days=retention_days)
        keep = [d for d in self._deltas if d.timestamp >= cutoff]
        n = len(self._deltas) - len(keep)
        self._deltas = keep
        return n
