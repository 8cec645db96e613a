"""Summary-hash commitment of a session's Merkle root.

Parity target: reference ``audit/commitment.py:15-77``: an in-memory
``session → record`` map with ``committed_to="local"``; ``verify`` compares the
stored root; ``queue_for_batch`` / ``flush_batch`` drain a queue.

Multi-GPU: under session sharding each rank commits its own sessions; the
cross-rank view (collective X06, an all-gather of (session slot, 32-byte root,
delta count)) is assembled by
:func:`agent_hypervisor_amd.parallel.collectives.allgather_commitments` at flush.
"""

from __future__ import annotations

from dataclasses import dataclass, field
from datetime import datetime
from typing import Optional

from hypervisor._clock import now as _now


@dataclass
class CommitmentRecord:
    session_id: str
    merkle_root: str
    participant_dids: list[str]
    delta_count: int
    committed_at: datetime = field(default_factory=_now)
    blockchain_tx_id: Optional[str] = None
    committed_to: str = "local"


class CommitmentEngine:
    def __init__(self) -> None:
        self._commitments: dict[str, CommitmentRecord] = {}
        self._batch_queue: list[CommitmentRecord] = []

    def commit(
        self,
        session_id: str,
        merkle_root: str,
        participant_dids: list[str],
        delta_count: int,
    ) -> CommitmentRecord:
        rec = CommitmentRecord(session_id, merkle_root, participant_dids, delta_count)
        self._commitments[session_id] = rec
        return rec

    def verify(self, session_id: str, expected_root: str) -> bool:
        rec = self._commitments.get(session_id)
        return rec is not None and rec.merkle_root == expected_root

    def queue_for_batch(self, record: CommitmentRecord) -> None:
        self._batch_queue.append(record)

    def flush_batch(self) -> list[CommitmentRecord]:
        out, self._batch_queue = self._batch_queue, []
        return out

    def get_commitment(self, session_id: str) -> Optional[CommitmentRecord]:
        return self._commitments.get(session_id)

    @property
    def commitment_count(self) -> int:
        return len(self._commitments)

    def all_commitments(self) -> list[CommitmentRecord]:
        return list(self._commitments.values())
