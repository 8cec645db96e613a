"""Shared Session Object: the lifecycle owner of one multi-agent session.

Parity target: reference ``session/__init__.py:20-191``.

Lifecycle guards (``_assert_state``)::

    begin_handshake  CREATED                 -> HANDSHAKING
    activate         HANDSHAKING (≥1 joined) -> ACTIVE
    join             HANDSHAKING | ACTIVE
    terminate        ACTIVE | HANDSHAKING    -> TERMINATING
    archive          TERMINATING             -> ARCHIVED
    snapshot/restore ACTIVE

Join admission (in order): duplicate DID, capacity over *active* participants,
σ_eff floor — the floor is waived for Ring-3 (sandbox) joins.

In the batched device engine the same lifecycle is a u8 state column with the
transition table in ``csrc/include/ahv/semantics.h`` (``session_transition``).
"""

from __future__ import annotations

from typing import Any, Optional

from agent_hypervisor_amd._native import C as _C
from hypervisor._clock import now as _now
from hypervisor.models import (
    ConsistencyMode,
    ExecutionRing,
    SessionConfig,
    SessionParticipant,
    SessionState,
)
from hypervisor.session.sso import SessionVFS

_uuid4 = _C.uuid4
_S = SessionState


class SessionLifecycleError(Exception):
    """A lifecycle operation was attempted from a state that does not allow it."""


class SessionParticipantError(Exception):
    """Join/leave/lookup failure for a participant."""


class SharedSessionObject:
    """A shared multi-agent session: participants, VFS substrate, lifecycle."""

    def __init__(
        self,
        config: SessionConfig,
        creator_did: str,
        session_id: Optional[str] = None,
    ):
        self.session_id = session_id or _uuid4("session:")
        self.creator_did = creator_did
        self.config = config
        self.state = _S.CREATED
        self.consistency_mode = config.consistency_mode
        self._participants: dict[str, SessionParticipant] = {}
        self.vfs_namespace = "/sessions/" + self.session_id
        self.vfs = SessionVFS(self.session_id, namespace=self.vfs_namespace)
        self._vfs_snapshots: dict[str, Any] = {}
        self.created_at = _now()
        self.terminated_at = None

    # -- participants -----------------------------------------------------
    @property
    def participants(self) -> list[SessionParticipant]:
        return [p for p in self._participants.values() if p.is_active]

    @property
    def participant_count(self) -> int:
        n = 0
        for p in self._participants.values():
            if p.is_active:
                n += 1
        return n

    # -- lifecycle --------------------------------------------------------
    def snapshot(self, parts: bool = True):
        """A :class:`hypervisor.session.snapshot.SessionSnapshot` of this session
        (the device session reads it in one round trip)."""
        from hypervisor.session.snapshot import SessionSnapshot

        return SessionSnapshot.of(self, parts)

    def _assert_state(self, *allowed: SessionState) -> None:
        if self.state not in allowed:
            raise SessionLifecycleError(
                f"Operation not allowed in state {self.state.value}. "
                f"Allowed: {[s.value for s in allowed]}"
            )

    def begin_handshake(self) -> None:
        if self.state is not _S.CREATED:
            self._assert_state(_S.CREATED)
        self.state = _S.HANDSHAKING

    def activate(self) -> None:
        if self.state is not _S.HANDSHAKING:
            self._assert_state(_S.HANDSHAKING)
        if not self._participants:
            raise SessionLifecycleError("Cannot activate session with no participants")
        self.state = _S.ACTIVE

    def join(
        self,
        agent_did: str,
        sigma_raw: float = 0.0,
        sigma_eff: float = 0.0,
        ring: ExecutionRing = ExecutionRing.RING_3_SANDBOX,
    ) -> SessionParticipant:
        if self.state is not _S.HANDSHAKING and self.state is not _S.ACTIVE:
            self._assert_state(_S.HANDSHAKING, _S.ACTIVE)
        if agent_did in self._participants:
            raise SessionParticipantError(f"Agent {agent_did} already in session")
        cfg = self.config
        if self.participant_count >= cfg.max_participants:
            raise SessionParticipantError(f"Session at capacity ({cfg.max_participants})")
        if ring != ExecutionRing.RING_3_SANDBOX and sigma_eff < cfg.min_sigma_eff:
            raise SessionParticipantError(
                f"σ_eff {sigma_eff:.2f} below minimum {cfg.min_sigma_eff:.2f}"
            )
        p = SessionParticipant(agent_did=agent_did, ring=ring, sigma_raw=sigma_raw, sigma_eff=sigma_eff)
        self._participants[agent_did] = p
        return p

    def leave(self, agent_did: str) -> None:
        self.get_participant(agent_did).is_active = False

    def get_participant(self, agent_did: str) -> SessionParticipant:
        p = self._participants.get(agent_did)
        if p is None:
            raise SessionParticipantError(f"Agent {agent_did} not in session")
        return p

    def update_ring(self, agent_did: str, new_ring: ExecutionRing) -> None:
        self.get_participant(agent_did).ring = new_ring

    def force_consistency_mode(self, mode: ConsistencyMode) -> None:
        self.consistency_mode = mode

    def terminate(self) -> None:
        if self.state is not _S.ACTIVE and self.state is not _S.HANDSHAKING:
            self._assert_state(_S.ACTIVE, _S.HANDSHAKING)
        self.state = _S.TERMINATING
        self.terminated_at = _now()

    def archive(self) -> None:
        if self.state is not _S.TERMINATING:
            self._assert_state(_S.TERMINATING)
        self.state = _S.ARCHIVED

    # -- VFS snapshots ------------------------------------------------------
    def create_vfs_snapshot(self, snapshot_id: Optional[str] = None) -> str:
        self._assert_state(_S.ACTIVE)
        sid = self.vfs.create_snapshot(snapshot_id)
        self._vfs_snapshots[sid] = {
            "created_at": _now().isoformat(),
            "participant_states": {
                did: {"ring": p.ring.value, "sigma_eff": p.sigma_eff}
                for did, p in self._participants.items()
            },
        }
        return sid

    def restore_vfs_snapshot(self, snapshot_id: str, agent_did: str) -> None:
        self._assert_state(_S.ACTIVE)
        self.vfs.restore_snapshot(snapshot_id, agent_did)

    def __repr__(self) -> str:
        return (
            f"SharedSessionObject(id={self.session_id!r}, state={self.state.value}, "
            f"participants={self.participant_count}, mode={self.consistency_mode.value})"
        )


__all__ = [
    "SharedSessionObject",
    "SessionLifecycleError",
    "SessionParticipantError",
    "SessionVFS",
]
