"""Session snapshots: one consistent read of a session row.

List and aggregate views (REST ``/api/v1/sessions``, ``/api/v1/stats``, the
dashboard, the sharded views) read every session; on a device-backed hypervisor
:func:`hypervisor._device.snapshots` fills these from one batched store command
instead of one device round trip per field per session.
"""

from __future__ import annotations


class SessionSnapshot:
    """One consistent read of a session row (state, counts, participants): what
    the list / aggregate views need, without a device round trip per field."""

    __slots__ = ("session_id", "state", "consistency_mode", "participant_count", "created_at", "terminated_at",
                 "delta_count", "participants", "creator_did", "committed_at", "commit_count", "merkle_root",
                 "commit_dids")

    @classmethod
    def of(cls, sso, parts: bool = False) -> "SessionSnapshot":
        """Host engines: read the live object."""
        s = cls()
        s.session_id = sso.session_id
        s.state = sso.state
        s.consistency_mode = sso.consistency_mode
        s.participant_count = sso.participant_count
        s.created_at = sso.created_at
        s.terminated_at = sso.terminated_at
        s.creator_did = sso.creator_did
        s.delta_count = None
        s.participants = list(sso.participants) if parts else None
        s.committed_at = s.commit_count = s.merkle_root = s.commit_dids = None  # host: ask the CommitmentEngine
        return s
