"""DID transaction-history verification at handshake time.

Parity target: reference ``verification/history.py:16-161``.

* Results are cached per agent and the cache always wins (``cached=True``).
* No history, or fewer than 5 records → PROBATIONARY; otherwise VERIFIED unless
  the history is inconsistent (duplicate summary hash, non-monotonic
  timestamps, empty or < 16-char hash) → SUSPICIOUS.
* ``is_trustworthy`` ⇔ VERIFIED or PROBATIONARY.

``Hypervisor.join_session`` forwards an optional declared history (the reference
never passed one, so its sandbox override was unreachable — Q23).
"""

from __future__ import annotations

from dataclasses import dataclass, field
from datetime import datetime
from enum import Enum
from typing import Optional

from hypervisor._clock import now as _now


class VerificationStatus(str, Enum):
    VERIFIED = "verified"
    PROBATIONARY = "probationary"
    SUSPICIOUS = "suspicious"
    UNREACHABLE = "unreachable"
    UNKNOWN = "unknown"


@dataclass
class TransactionRecord:
    session_id: str
    summary_hash: str
    timestamp: datetime
    participant_count: int = 0


@dataclass
class VerificationResult:
    agent_did: str
    status: VerificationStatus
    transactions_checked: int
    transactions_found: int
    inconsistencies: list[str] = field(default_factory=list)
    verified_at: datetime = field(default_factory=_now)
    cached: bool = False

    @property
    def is_trustworthy(self) -> bool:
        return self.status in (VerificationStatus.VERIFIED, VerificationStatus.PROBATIONARY)


class TransactionHistoryVerifier:
    REQUIRED_HISTORY_DEPTH = 5
    MIN_HASH_LENGTH = 16

    def __init__(self) -> None:
        self._cache: dict[str, VerificationResult] = {}

    def verify(
        self,
        agent_did: str,
        declared_history: Optional[list[TransactionRecord]] = None,
    ) -> VerificationResult:
        hit = self._cache.get(agent_did)
        if hit is not None:
            hit.cached = True
            return hit
        n = len(declared_history) if declared_history else 0
        if n == 0:
            res = VerificationResult(
                agent_did, VerificationStatus.PROBATIONARY, 0, 0, ["No transaction history available"]
            )
        elif n < self.REQUIRED_HISTORY_DEPTH:
            res = VerificationResult(
                agent_did,
                VerificationStatus.PROBATIONARY,
                n,
                n,
                [f"Only {n} transactions (need {self.REQUIRED_HISTORY_DEPTH})"],
            )
        else:
            issues = self._check_consistency(declared_history)
            res = VerificationResult(
                agent_did,
                VerificationStatus.SUSPICIOUS if issues else VerificationStatus.VERIFIED,
                n,
                n,
                issues,
            )
        self._cache[agent_did] = res
        return res

    def clear_cache(self, agent_did: Optional[str] = None) -> None:
        if agent_did:
            self._cache.pop(agent_did, None)
        else:
            self._cache.clear()

    def _check_consistency(self, history: list[TransactionRecord]) -> list[str]:
        issues: list[str] = []
        first_seen: dict[str, str] = {}
        for tx in history:
            prior = first_seen.get(tx.summary_hash)
            if prior is not None:
                issues.append(f"Duplicate hash in sessions {prior} and {tx.session_id}")
            first_seen[tx.summary_hash] = tx.session_id
        for prev, cur in zip(history, history[1:]):
            if cur.timestamp < prev.timestamp:
                issues.append(f"Non-monotonic timestamps: {cur.session_id} predates {prev.session_id}")
        for tx in history:
            if not tx.summary_hash or len(tx.summary_hash) < self.MIN_HASH_LENGTH:
                issues.append(f"Invalid hash in session {tx.session_id}")
        return issues
