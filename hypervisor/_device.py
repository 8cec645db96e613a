"""Device-backed engines: the public API over the gfx950 state store.

``Hypervisor(device="cuda")`` (or ``"cpu"`` for the host twin of the same
command processor) swaps its stateful engines for the classes below.  Each is a
subclass of the host engine it replaces — same methods, same exceptions and
messages — but holds no governance state of its own: every read and write is a
command against :class:`agent_hypervisor_amd.models.store.GovernanceStore`
(``csrc/include/ahv/store.h``):

=============================  ===============================================
engine                         device commands (kernel ids)
=============================  ===============================================
:class:`DeviceSession`         lifecycle FSM, join admission + ring gate (K01)
:class:`DeviceDeltaEngine`     chain-linked SHA-256 capture (K08), Merkle root
                               (K09), verification of presented records (K10)
:class:`DeviceVouchingEngine`  vouch admission with cycle/exposure checks (K05),
                               σ_eff (K03), exposure (K04), bond release (K07)
:class:`DeviceSlashingEngine`  slash + cascade (K06)
:class:`DeviceSagaOrchestrator` step / saga FSM (K13), compensation plan (K14)
:class:`DeviceCommitmentEngine` commitments written by the terminate command
=============================  ===============================================

What stays on the host is what is not governance state: interned-id lookups
(DIDs, session/vouch/saga ids → rows), the Python objects callers hand in
(executors, results, VFS file contents) and error-message formatting.  Returned
records (participants, vouch records, deltas, sagas) are *views*: their state
fields are read from the device when accessed.
"""

from __future__ import annotations

import asyncio
import os
import struct
from datetime import datetime, timedelta
from typing import Any, Callable, Optional

import numpy as np

from agent_hypervisor_amd._native import C as _C
from agent_hypervisor_amd.models import store as _st
from agent_hypervisor_amd.models.store import GovernanceStore, bitsd, dbits
from hypervisor import config as _cfg
from hypervisor._clock import from_us, now as _now, now_us as _now_us, to_us
from hypervisor.audit.commitment import CommitmentEngine, CommitmentRecord
from hypervisor.audit.delta import DeltaEngine, SemanticDelta, VFSChange, _payload_json
from hypervisor.liability.slashing import SlashingEngine, SlashResult, VoucherClip
from hypervisor.liability.vouching import VouchingEngine, VouchingError, VouchRecord
from hypervisor.models import ConsistencyMode, ExecutionRing, SessionConfig, SessionParticipant, SessionState
from hypervisor.saga._timeout import await_with_timeout
from hypervisor.saga.orchestrator import SagaOrchestrator, SagaTimeoutError
from hypervisor.saga.state_machine import (
    SAGA_TRANSITIONS,
    STEP_TRANSITIONS,
    Saga,
    SagaState,
    SagaStateError,
    SagaStep,
    StepState,
)
from hypervisor.session import SessionLifecycleError, SessionParticipantError, SharedSessionObject
from hypervisor.session.snapshot import SessionSnapshot
from hypervisor.session.sso import SessionVFS

_STATES = list(SessionState)
_S_CREATED, _S_HANDSHAKING, _S_ACTIVE = (_STATES.index(x) for x in (SessionState.CREATED, SessionState.HANDSHAKING,
                                                                   SessionState.ACTIVE))
# A/B switch: joins / activations / step transitions whose outcome the host already knows
# are posted without waiting for the device (verified later; GovernanceStore.post_checked)
_SPEC_LIFECYCLE = os.environ.get("AHV_SPEC_LIFECYCLE", "1") != "0"
# ... and a terminate whose Merkle root the host predicted from its SHA-NI digest
# predictions (K08/K09 on the host beside the device; the device's own root is what
# it commits, and it must equal the prediction)
# terminate awaits the device's Merkle root by default (the store is the authority);
# AHV_SPEC_TERMINATE=1 returns the host's SHA-NI prediction at once and checks the
# device's committed root afterwards (a divergence poisons the session)
_SPEC_TERMINATE = os.environ.get("AHV_SPEC_TERMINATE", "0") != "0"
# awaited terminates compare the device's root with the host's prediction (AHV_CHECK_TERMINATE=0: off)
_CHECK_TERMINATE = os.environ.get("AHV_CHECK_TERMINATE", "1") != "0"
_STEPS = list(StepState)
_STEP_IDX = {**{x: i for i, x in enumerate(_STEPS)}, **{x.value: i for i, x in enumerate(_STEPS)}}
_COMMITTED_IDX = _STEP_IDX[StepState.COMMITTED]
_SAGAS = list(SagaState)
_RINGS = list(ExecutionRing)
_MODE = {ConsistencyMode.EVENTUAL: 0, ConsistencyMode.STRONG: 1}
_MODES = [ConsistencyMode.EVENTUAL, ConsistencyMode.STRONG]
_NAN = dbits(float("nan"))


def _u64(v: int) -> int:
    return v & 0xFFFFFFFFFFFFFFFF


def _i64(v: int) -> int:
    v &= 0xFFFFFFFFFFFFFFFF
    return v - (1 << 64) if v >= 1 << 63 else v


_PACK8 = struct.Struct(">8I").pack


def _hex(words) -> str:
    """Hex of eight 32-bit digest words (one struct pack: ~10x the per-word format)."""
    try:
        return _PACK8(*words).hex()
    except struct.error:  # not eight words in range
        return "".join(f"{int(w) & 0xFFFFFFFF:08x}" for w in words)


def _words(hexstr: str) -> list[int]:
    return [int(hexstr[8 * k: 8 * k + 8], 16) for k in range(8)]


def _lifecycle(state_code: int, *allowed: SessionState) -> SessionLifecycleError:
    st = _STATES[state_code] if state_code < len(_STATES) else state_code
    val = st.value if isinstance(st, SessionState) else str(st)
    return SessionLifecycleError(f"Operation not allowed in state {val}. Allowed: {[s.value for s in allowed]}")


_STORE_BY_MODE: dict = {}


def _shared_store(mode: str) -> GovernanceStore:
    """The process-wide store of a ``Hypervisor(device=...)`` mode string (cached per
    string: one dict lookup per Hypervisor instead of a torch.device parse)."""
    st = _STORE_BY_MODE.get(mode)
    if st is None or getattr(st, "_closed", False):
        st = _STORE_BY_MODE[mode] = _st.shared_store(mode)
    return st


def _id_words(session_id: str, store: GovernanceStore) -> tuple:
    """(hi, lo) signed id words of a session row: the uuid's halves, or for an id
    that is not a uuid, 0 and a per-store serial."""
    u = session_id.rsplit(":", 1)[-1].replace("-", "")
    try:
        hi, lo = int(u[:16], 16), int(u[16:32], 16)
    except ValueError:
        hi = lo = 0
    if len(u) != 32 or not lo:  # not a uuid id: a per-store serial stands in for its id words
        hi, lo = 0, store.next_stamp()
    return _i64(hi), _i64(lo)


def _check(res: tuple, what: str) -> tuple:
    if res[0] in (_st.ST_BAD_ARG, _st.ST_SCRATCH) or res[0] >= 90:
        raise _st.StoreError(f"store command {what} failed with status {res[0]}")
    return res


# ------------------------------------------------------------------ sessions


class DeviceSession(SharedSessionObject):
    """A :class:`SharedSessionObject` whose lifecycle and participants live on the device."""

    def __init__(
        self,
        store: GovernanceStore,
        config: SessionConfig,
        creator_did: str,
        session_id: Optional[str] = None,
        handshake: bool = True,
        slot: Optional[int] = None,
        create: bool = True,
    ) -> None:
        self._store = store
        words = None
        if session_id is None:
            session_id, hi, lo = _C.uuid4_id("session:")  # the id and its row id words
            words = (hi, lo)
        self.session_id = session_id
        self.creator_did = creator_did
        self.config = config
        self.vfs_namespace = "/sessions/" + session_id
        self._vfs_snapshots: dict[str, Any] = {}
        self.slot = store.alloc("S") if slot is None else slot
        self._cseq = -1
        # Host mirror of the row's admission state (state code, agent id → active for every
        # participant row), valid while every change to the row goes through this object:
        # then join / activate outcomes are known before the device confirms them and are
        # posted without waiting (verified later, GovernanceStore.post_checked).  None: unknown.
        self._m_state: Optional[int] = None
        self._m_rows: Optional[dict] = None
        self._m_active = 0
        if create and _SPEC_LIFECYCLE:
            self._m_state = _S_HANDSHAKING if handshake else _S_CREATED
            self._m_rows = {}
            self._m_cfg = (int(config.max_participants), float(config.min_sigma_eff))  # what the row holds
        self._stamp = 0  # creation stamp this object sent (0: not created here)
        self._poisoned: Optional[Exception] = None  # a speculated post of this session the device refused
        if create:
            if words is None:
                words = _id_words(session_id, store)
            hi, lo = words
            # the creation stamp later posts carry is the row's id words (row_stamp in
            # store.h), not a clock value: creates in one µs / under a pinned clock differ
            args = [
                self.slot, store.agent_id(creator_did), _now_us(), _MODE[config.consistency_mode],
                int(config.max_participants), dbits(config.min_sigma_eff), int(bool(config.enable_audit)),
                hi, lo, 0 if handshake else 1,
            ]
            if self._m_state is not None and lo:
                # posted and verified later: the join / activate that follow carry the stamp,
                # so a row holding another session (a refused create) refuses them on the device
                self._stamp = lo
                slot = self.slot
                store.post_expect(_st.OP_SESS_CREATE, args, _OK, (self, _create_refused, slot))
            else:
                self._cseq = store.post(_st.OP_SESS_CREATE, args)

    @property
    def vfs(self) -> SessionVFS:  # type: ignore[override]
        """The session's VFS, built on first use (most sessions never touch it)."""
        v = self.__dict__.get("_vfs")
        if v is None:
            v = self.__dict__["_vfs"] = SessionVFS(self.session_id, namespace=self.vfs_namespace)
        return v

    @vfs.setter
    def vfs(self, v: SessionVFS) -> None:
        self.__dict__["_vfs"] = v

    def vfs_if_built(self) -> Optional[SessionVFS]:
        """The VFS if anything has used it, else None (an unused VFS holds no files)."""
        return self.__dict__.get("_vfs")

    def __del__(self) -> None:
        # the row stays allocated while this view (or a delta engine / saga built
        # on it) exists; afterwards the store may reclaim it.  The view is detached
        # first: in cyclic garbage another finaliser (Hypervisor.close) may still
        # see this object and must not release the row a second time.
        try:
            st, self._store = self._store, CLOSED
            st.release("S", self.slot)
        except Exception:
            pass

    # -- speculation failures (GovernanceStore.post_checked) -----------------------
    def _spec_failed(self, exc: Exception) -> None:
        """The device disagreed with a prediction this session posted: from now on
        every operation of this session raises it (the first one is kept)."""
        if self._poisoned is None:
            self._poisoned = exc
        self._m_forget()  # the mirror is wrong: nothing more is speculated for this row

    def _guard(self) -> None:
        """Raise this session's speculation failure, if any (after checking the
        predictions whose results are in)."""
        self._store.verify_deferred()
        if self._poisoned is not None:
            raise self._poisoned

    def _created(self) -> None:
        """Raise if the device refused the create (the slot was not free)."""
        q = self._cseq
        if q >= 0:
            self._cseq = -1
            r = self._store.result(q, 2)
            if r is not None and r[0]:
                raise _st.StoreError(f"device refused to create session {self.session_id} in row {self.slot} "
                                     f"(row state {r[1]}): allocator invariant violated")

    # -- device reads -----------------------------------------------------------
    def _read(self, with_parts: bool = False):
        r = self._store.call(_st.OP_SESS_READ, [self.slot, 0], 36)
        parts = []
        if with_parts and r[3]:
            raw = self._store.bulk(0, 40 * r[3])
            for k in range(r[3]):
                a, fl, sr, se, j = struct.unpack_from("<qQddq", raw, 40 * k)
                parts.append((a, fl & 0xFF, (fl >> 8) & 1, sr, se, j))  # bit 8 P_ACTIVE, bit 9 P_COMMITTED
        return r, parts

    def _participant(self, row) -> SessionParticipant:
        a, ring, active, sr, se, j = row
        return SessionParticipant(
            agent_did=self._store.did(a), ring=_RINGS[ring], sigma_raw=sr, sigma_eff=se,
            joined_at=from_us(j), is_active=bool(active),
        )

    @property
    def state(self) -> SessionState:
        return _STATES[self._store.call(_st.OP_SESS_READ, [self.slot, 0], 2)[1]]

    @state.setter
    def state(self, value) -> None:  # the base class never assigns on this path
        raise AttributeError("device session state changes only through lifecycle methods")

    @property
    def consistency_mode(self) -> ConsistencyMode:
        return _MODES[self._store.call(_st.OP_SESS_READ, [self.slot, 0], 3)[2]]

    @consistency_mode.setter
    def consistency_mode(self, mode) -> None:
        self.force_consistency_mode(mode)

    @property
    def created_at(self) -> datetime:
        return from_us(self._store.call(_st.OP_SESS_READ, [self.slot, 0], 6)[5])

    @created_at.setter
    def created_at(self, v) -> None:
        raise AttributeError("created_at is recorded by the device")

    @property
    def terminated_at(self) -> Optional[datetime]:
        t = self._store.call(_st.OP_SESS_READ, [self.slot, 0], 7)[6]
        return from_us(t) if t else None

    @terminated_at.setter
    def terminated_at(self, v) -> None:
        raise AttributeError("terminated_at is recorded by the device")

    @property
    def _participants(self) -> dict[str, SessionParticipant]:
        _, parts = self._read(True)
        return {p.agent_did: p for p in (self._participant(r) for r in parts)}

    @property
    def participants(self) -> list[SessionParticipant]:
        _, parts = self._read(True)
        return [self._participant(r) for r in parts if r[2]]

    @property
    def participant_count(self) -> int:
        return self._store.call(_st.OP_SESS_READ, [self.slot, 0], 5)[4]

    def snapshot(self, parts: bool = True):
        """Every field of the session row (and its participants) in one batched
        read — the form for callers that need several fields at once (each
        property above is its own device round trip)."""
        return snapshots(self._store, [self], parts)[0]

    # -- lifecycle ---------------------------------------------------------------
    def begin_handshake(self) -> None:
        r = self._store.call(_st.OP_SESS_HANDSHAKE, [self.slot], 2)
        if r[0]:
            raise _lifecycle(r[1], SessionState.CREATED)
        if self._m_state is not None:
            self._m_state = _S_HANDSHAKING

    def _activate_known_ok(self) -> bool:
        return self._m_state == _S_HANDSHAKING and bool(self._m_rows)

    def _activate_speculated(self) -> None:
        """The row is HANDSHAKING with ≥ 1 participant row: the device will accept."""
        slot = self.slot
        self._store.post_expect(_st.OP_SESS_ACTIVATE, [slot, self._stamp], _OK, (self, _activate_refused, slot))
        self._m_state = _S_ACTIVE

    def activate(self) -> None:
        self._guard()
        if self._cseq >= 0:
            self._created()
        if self._activate_known_ok():
            return self._activate_speculated()
        self._activated(self._store.call(_st.OP_SESS_ACTIVATE, [self.slot, self._stamp], 2))
        if self._m_state is not None:
            self._m_state = _S_ACTIVE

    async def activate_async(self) -> None:
        self._guard()
        if self._cseq >= 0:
            self._created()
        if self._activate_known_ok():
            return self._activate_speculated()
        self._activated(await self._store.call_async(_st.OP_SESS_ACTIVATE, [self.slot, self._stamp], 2))
        if self._m_state is not None:
            self._m_state = _S_ACTIVE

    @staticmethod
    def _activated(r: tuple) -> None:
        if r[0] == _st.ST_BAD_STATE:
            raise _lifecycle(r[1], SessionState.HANDSHAKING)
        if r[0] == 3:
            raise SessionLifecycleError("Cannot activate session with no participants")
        if r[0] == 4:
            raise _st.StoreError("activate: the row holds another session (its create was refused)")
        _check(r, "activate")

    def _join_args(self, agent_did: str, sigma_raw: float, sigma_eff: float, flags: int, ring: int) -> list:
        self._guard()
        if self._cseq >= 0:
            self._created()
        return [self.slot, self._store.agent_id(agent_did), dbits(sigma_raw), dbits(sigma_eff), flags, ring,
                _now_us(), self._stamp]

    def _join(self, agent_did: str, sigma_raw: float, sigma_eff: float, flags: int, ring: int) -> int:
        args = self._join_args(agent_did, sigma_raw, sigma_eff, flags, ring)
        if not flags & 2:
            got = self._join_speculated(args, sigma_eff, bool(flags & 1))
            if got is not None:
                return got
        r = self._store.call(_st.OP_SESS_JOIN, args, 6)
        return self._mirror_join(args[1], self._joined(r, agent_did, sigma_eff))

    def _join_speculated(self, args: list, sigma_eff: float, trustworthy: bool) -> Optional[int]:
        """The ring of a join the device will certainly admit (posted without waiting),
        or None: the outcome is not known here (refusals always take the awaited path,
        so the device's own error reaches the caller)."""
        rows = self._m_rows
        if self._m_state is None or rows is None or len(rows) >= self._store.caps["P"]:
            return None
        aid = args[1]
        maxpart, minsig = self._m_cfg
        code, ring = _C.join_predict(self._m_state, aid in rows, self._m_active, maxpart, float(sigma_eff), minsig,
                                     trustworthy)
        if code:
            return None
        slot = self.slot
        self._store.post_expect(_st.OP_SESS_JOIN, args, (0, int(ring)), (self, _join_diverged, slot))
        rows[aid] = True
        self._m_active += 1
        return ring

    def _mirror_join(self, aid: int, ring: int) -> int:
        if self._m_rows is not None:
            self._m_rows[aid] = True
            self._m_active += 1
        return ring

    async def join_gated_async(self, agent_did: str, sigma_raw: float, sigma_eff: float,
                               trustworthy: bool) -> ExecutionRing:
        """:meth:`join_gated` without blocking the event loop on the device round trip."""
        args = self._join_args(agent_did, sigma_raw, sigma_eff, 1 if trustworthy else 0, 0)
        got = self._join_speculated(args, sigma_eff, trustworthy)
        if got is not None:
            return _RINGS[got]
        r = await self._store.call_async(_st.OP_SESS_JOIN, args, 6)
        return _RINGS[self._mirror_join(args[1], self._joined(r, agent_did, sigma_eff))]

    def _joined(self, r: tuple, agent_did: str, sigma_eff: float) -> int:
        code = r[0]
        if code == 0:
            return r[1]
        if code == 1:
            raise _lifecycle(r[2], SessionState.HANDSHAKING, SessionState.ACTIVE)
        if code == 2:
            raise SessionParticipantError(f"Agent {agent_did} already in session")
        if code in (3, 5):
            raise SessionParticipantError(f"Session at capacity ({self.config.max_participants})")
        if code == 4:
            raise SessionParticipantError(f"σ_eff {sigma_eff:.2f} below minimum {bitsd(r[5]):.2f}")
        if code == 6:
            raise _st.StoreError("join: the row holds another session (its create was refused)")
        raise _st.StoreError(f"join failed with status {code}")

    def join(self, agent_did: str, sigma_raw: float = 0.0, sigma_eff: float = 0.0,
             ring: ExecutionRing = ExecutionRing.RING_3_SANDBOX) -> SessionParticipant:
        self._join(agent_did, sigma_raw, sigma_eff, 2, int(ring))
        return SessionParticipant(agent_did=agent_did, ring=ring, sigma_raw=sigma_raw, sigma_eff=sigma_eff)

    def join_gated(self, agent_did: str, sigma_raw: float, sigma_eff: float, trustworthy: bool) -> ExecutionRing:
        """Join with the ring computed on the device (K01 ring gate); returns the ring."""
        return _RINGS[self._join(agent_did, sigma_raw, sigma_eff, 1 if trustworthy else 0, 0)]

    def leave(self, agent_did: str) -> None:
        self._guard()
        aid = self._store.agent_id(agent_did)
        r = self._store.call(_st.OP_SESS_LEAVE, [self.slot, aid], 1)
        if r[0]:
            raise SessionParticipantError(f"Agent {agent_did} not in session")
        rows = self._m_rows
        if rows is not None and rows.get(aid):
            rows[aid] = False
            self._m_active -= 1

    def get_participant(self, agent_did: str) -> SessionParticipant:
        p = self._participants.get(agent_did)
        if p is None:
            raise SessionParticipantError(f"Agent {agent_did} not in session")
        return p

    def update_ring(self, agent_did: str, new_ring: ExecutionRing) -> None:
        r = self._store.call(_st.OP_SESS_UPDATE_RING, [self.slot, self._store.agent_id(agent_did), int(new_ring)], 1)
        if r[0]:
            raise SessionParticipantError(f"Agent {agent_did} not in session")

    def set_sigma(self, agent_did: str, sigma_eff: float, ring: Optional[ExecutionRing] = None) -> None:
        args = [self.slot, self._store.agent_id(agent_did), dbits(sigma_eff), 1 if ring is not None else 0,
                int(ring) if ring is not None else 0]
        if self._store.call(_st.OP_SESS_SET_SIGMA, args, 1)[0]:
            raise SessionParticipantError(f"Agent {agent_did} not in session")

    def force_consistency_mode(self, mode: ConsistencyMode) -> None:
        self._store.post(_st.OP_SESS_SET_MODE, [self.slot, _MODE[ConsistencyMode(mode)]])

    def _m_forget(self) -> None:
        """The row leaves the states joins/activation can change: stop mirroring it."""
        self._m_state = None
        self._m_rows = None

    def terminate(self) -> None:
        self._guard()
        self._m_forget()
        r = self._store.call(_st.OP_SESS_TERMINATE, [self.slot, _now_us()], 2)
        if r[0]:
            raise _lifecycle(r[1], SessionState.ACTIVE, SessionState.HANDSHAKING)

    def archive(self) -> None:
        self._guard()
        self._m_forget()
        r = self._store.call(_st.OP_SESS_ARCHIVE, [self.slot], 2)
        if r[0]:
            raise _lifecycle(r[1], SessionState.TERMINATING)

    def create_vfs_snapshot(self, snapshot_id: Optional[str] = None) -> str:
        r, parts = self._read(True)
        if r[1] != 2:
            raise _lifecycle(r[1], SessionState.ACTIVE)
        sid = self.vfs.create_snapshot(snapshot_id)
        self._vfs_snapshots[sid] = {
            "created_at": _now().isoformat(),
            "participant_states": {
                self._store.did(p[0]): {"ring": p[1], "sigma_eff": p[4]} for p in parts
            },
        }
        return sid

    def restore_vfs_snapshot(self, snapshot_id: str, agent_did: str) -> None:
        st = self.state
        if st is not SessionState.ACTIVE:
            raise _lifecycle(_STATES.index(st), SessionState.ACTIVE)
        self.vfs.restore_snapshot(snapshot_id, agent_did)

    def __repr__(self) -> str:
        r, _ = self._read(False)
        return (
            f"SharedSessionObject(id={self.session_id!r}, state={_STATES[r[1]].value}, "
            f"participants={r[4]}, mode={_MODES[r[2]].value}, device_slot={self.slot})"
        )


# ------------------------------------------------------------------ audit


class DeviceDelta(SemanticDelta):
    """A captured delta whose digest and parent link are held by the device chain.

    It refers to the store, not to its engine: the engine lists its deltas, and a
    back-reference would make every chain a reference cycle that only the cyclic
    collector frees — the rows of a dropped session would then wait for a
    ``gc.collect()`` instead of being released when the last reference goes."""

    def __init__(self, engine: "DeviceDeltaEngine", delta_id, turn_id, session_id, agent_did, timestamp, changes,
                 prev: Optional["DeviceDelta"]) -> None:
        self.__dict__.update(
            delta_id=delta_id, turn_id=turn_id, session_id=session_id, agent_did=agent_did, timestamp=timestamp,
            changes=changes, _store=engine._store, _prev=prev, _dev_hash=None, _hash_override=None,
            _parent_override=None, _didx=-1, _poff=-1, _plen=0, _seq=-1, _dirty=False, _pred=None, _tsu=0,
        )

    _FIELDS = frozenset(("delta_id", "turn_id", "session_id", "agent_did", "timestamp", "changes"))

    def __setattr__(self, k, v) -> None:
        # an edit of a hashed field after capture: the view no longer shows what
        # the device holds, so audits of this chain re-render the views
        if k in DeviceDelta._FIELDS:
            self.__dict__[k] = v
            self.__dict__["_dirty"] = True
        else:
            object.__setattr__(self, k, v)

    def device_hash(self) -> str:
        """The digest the device computed for this delta (K08)."""
        h = self.__dict__["_dev_hash"]
        if h is None:
            h = _resolve(self._store, self)
        return h

    @property
    def delta_hash(self) -> str:  # type: ignore[override]
        o = self.__dict__["_hash_override"]
        return o if o is not None else self.device_hash()

    @delta_hash.setter
    def delta_hash(self, v: str) -> None:
        self.__dict__["_hash_override"] = v
        self.__dict__["_dirty"] = True

    @property
    def parent_hash(self) -> Optional[str]:  # type: ignore[override]
        o = self.__dict__["_parent_override"]
        if o is not None:
            return None if o is _NULL else o
        prev = self.__dict__["_prev"]
        return prev.device_hash() if prev is not None else None

    @parent_hash.setter
    def parent_hash(self, v: Optional[str]) -> None:
        self.__dict__["_parent_override"] = _NULL if v is None else v
        self.__dict__["_dirty"] = True

    def compute_hash(self) -> str:
        self.delta_hash = _host_digest(self)
        return self.delta_hash

    def record(self) -> bytes:
        """The device-held canonical-JSON record (exact hashed bytes)."""
        return self._store.payload(self._poff, self._plen)

    def __repr__(self) -> str:
        return f"DeviceDelta(delta_id={self.delta_id!r}, turn_id={self.turn_id}, session_id={self.session_id!r})"


_NULL = object()


def _render(d) -> bytes:
    b = _C.delta_payload(d)
    return b if b is not None else _payload_json(d).encode()


def _host_digest(d) -> str:
    import hashlib

    return hashlib.sha256(_render(d)).hexdigest()


class DeviceDeltaEngine(DeltaEngine):
    """Audit chain of one device session: the device links, hashes and roots it."""

    def __init__(self, store: GovernanceStore, slot: int, session_id: str,
                 owner: Optional[DeviceSession] = None) -> None:
        self._store = store
        self.slot = slot
        self.session_id = session_id
        self._owner = owner  # keeps the session row allocated while the chain is reachable
        self._deltas: list[DeviceDelta] = []
        self._rows: list[int] = []  # every delta row this chain owns (pruned views included)
        self._turn_counter = 0

    def __del__(self) -> None:
        try:
            rows, self._rows = self._rows, []
            st, self._store = self._store, CLOSED
            if rows:
                st.release_many("D", rows)
        except Exception:
            pass

    def capture(self, agent_did: str, changes: list[VFSChange], delta_id: Optional[str] = None) -> DeviceDelta:
        turn = self._turn_counter + 1
        ts = _now()
        prev = self._deltas[-1] if self._deltas else None
        d = DeviceDelta(self, delta_id or f"delta:{turn}", turn, self.session_id, agent_did, ts, changes, prev)
        # the device's digest, predicted on the host from the same bytes and the
        # previous prediction (terminate then needs no wait for the hash engine)
        parent = prev.__dict__["_pred"] if prev is not None else None
        tsu = to_us(ts)
        didx, off, ln, seq, pred = self._store.capture(self.slot, turn, tsu, d, parent)
        if didx < 0:  # field types the native renderer defers to json.dumps
            raw = _payload_json(_NullParent(d)).encode()
            at = raw.index(b'"parent_hash": null') + len(b'"parent_hash": ')
            didx, off, ln, seq, pred = self._store.capture_bytes(self.slot, turn, tsu, raw, at, parent)
        self._rows.append(didx)
        d.__dict__.update(_didx=didx, _poff=off, _plen=ln, _seq=seq, _pred=pred, _tsu=tsu)
        self._turn_counter = turn
        self._deltas.append(d)
        return d

    def _resolve(self, d: DeviceDelta) -> str:
        return _resolve(self._store, d)

    def _indices(self) -> list[int]:
        return [d._didx for d in self._deltas]

    def compute_merkle_root(self) -> Optional[str]:
        if not self._deltas:
            return None
        n, off, inl = self._store.index_args(self._indices())
        r = _check(self._store.call(_st.OP_DELTA_MERKLE, [self.slot, n, off], 10, inl), "merkle")
        return _hex(r[2:10]) if r[1] else None

    def verify_chain(self) -> bool:
        if not self._deltas:
            return True
        parity = _cfg.parity_mode()
        blobs, recs = [], []
        pos = 0
        for d in self._deltas:
            raw = _render(d)
            blobs.append(raw)
            ph = d.parent_hash
            try:
                hw = _words(d.delta_hash)
            except (ValueError, TypeError):
                hw = [0] * 8
            try:
                pw = [0xFFFFFFFF] * 8 if ph is None else _words(ph)
            except (ValueError, TypeError):
                pw = [0] * 8
            recs.append((pos, len(raw), d._didx, hw, pw))
            pos += (len(raw) + 63) & ~63
        data = b"".join(b + b"\0" * (((len(b) + 63) & ~63) - len(b)) for b in blobs)
        base = self._store.stage(data)
        table = b"".join(
            struct.pack("<QQq8I8I", base + o, ln, didx, *hw, *pw) for (o, ln, didx, hw, pw) in recs
        )
        toff = self._store.stage(table)
        r = _check(self._store.call(_st.OP_DELTA_VERIFY, [self.slot, len(recs), toff, int(parity), 0], 3), "verify")
        if parity:  # reference verify rewrites every stored hash with the recomputed one (Q02)
            raw = self._store.bulk(0, 64 * len(recs))
            for i, d in enumerate(self._deltas):
                d.delta_hash = _hex(struct.unpack_from("<8Q", raw, 64 * i))
        return bool(r[1])

    @property
    def deltas(self) -> list[DeviceDelta]:
        return list(self._deltas)

    @property
    def turn_count(self) -> int:
        return self._turn_counter

    def export_records(self) -> list[dict]:
        return [{"payload": d.record().decode("ascii"), "delta_hash": d.device_hash()} for d in self._deltas]

    def prune_expired(self, retention_days: int) -> int:
        cutoff = _now() - timedelta(days=retention_days)
        keep = [d for d in self._deltas if d.timestamp >= cutoff]
        n = len(self._deltas) - len(keep)
        self._deltas = keep
        return n


def close_prediction(sso, de: "DeviceDeltaEngine", vsess: int, audit: bool, cutoff_us: int, check: bool = False):
    """(root, expired) the device's OP_SESS_CLOSE of this session will produce, when
    the host knows it: the row is mirrored in a state terminate accepts, the session
    holds no liability rows (their release is awaited), and every delta of the chain
    was captured here with a predicted digest.  None otherwise (the caller awaits).
    ``check``: the prediction an awaited terminate compares the device's root with
    (computed whatever AHV_SPEC_TERMINATE says, liability sessions included)."""
    if (not check and (not _SPEC_TERMINATE or vsess >= 0)) or sso._poisoned is not None:
        return None
    if sso._m_state != _S_ACTIVE and sso._m_state != _S_HANDSHAKING:
        return None
    ds = de._deltas
    if len(ds) != de._turn_counter:
        return None
    preds = [d.__dict__["_pred"] for d in ds]
    if None in preds:
        return None
    root = None
    if audit and preds:
        root = de._store._c.merkle_predict(preds)
        if root is None:
            return None
    expired = 0
    for d in ds:
        if d.__dict__["_tsu"] < cutoff_us:
            expired += 1
    return root, expired


def close_expect(root: Optional[str], expired: int) -> tuple:
    """The result words a speculated close must produce: status 0, the root flag and
    words (when a root is predicted), any release count, the GC count."""
    if root is None:
        return (0, None, None, None, None, None, None, None, None, None, None, expired)
    return (0, 1, *struct.unpack(">8I", bytes.fromhex(root)), None, expired)


def _close_diverged(slot: int, r: tuple) -> Exception:
    if r[0]:
        return _st.StoreError(f"speculated terminate of row {slot} refused by the device (status {r[0]})")
    return _st.StoreError(f"device Merkle root / GC count of row {slot} differs from the host prediction")


def _create_refused(slot: int, r: tuple) -> Exception:
    return _st.StoreError(f"device refused to create session in row {slot} (row state {r[1]}): "
                          "allocator invariant violated")


def _activate_refused(slot: int, r: tuple) -> Exception:
    return _st.StoreError(f"speculated activate of row {slot} refused by the device (status {r[0]})")


def _join_diverged(slot: int, r: tuple) -> Exception:
    return _st.StoreError(f"speculated join to row {slot} diverged from the device (status {r[0]})")


_OK = (0,)  # a speculated post's expected result: status 0


def _resolve(store: GovernanceStore, d: DeviceDelta) -> str:
    """The device digest of a captured delta (its capture result, or its arena row)."""
    r = store.result(d._seq, 9) if d._seq >= 0 else None
    if r is None:  # result slot recycled (or a restored / moved row): read the arena row
        n, off, inl = store.index_args([d._didx])
        store.call(_st.OP_DELTA_READ, [n, off, 0], 1, inl)
        raw = store.bulk(0, 96)
        r = (0,) + struct.unpack_from("<8Q", raw, 32)
    if r[0]:
        raise _st.StoreError(f"device capture of {d.delta_id} failed with status {r[0]}")
    h = _hex(r[1:9])
    d.__dict__["_dev_hash"] = h
    return h


class _NullParent:
    """Attribute proxy rendering a delta with a null parent (json.dumps fallback)."""

    def __init__(self, d) -> None:
        self._d = d

    def __getattr__(self, k):
        return None if k == "parent_hash" else getattr(self._d, k)


# ------------------------------------------------------------------ liability


class DeviceVouchRecord(VouchRecord):
    """A vouch edge view: identity on the host, bond state on the device."""

    def __init__(self, store: GovernanceStore, edge: int, vouch_id, voucher_did, vouchee_did, session_id, pct,
                 bonded, created_at, expiry, owner=None) -> None:
        self.__dict__.update(
            _store=store, edge=edge, vouch_id=vouch_id, voucher_did=voucher_did, vouchee_did=vouchee_did,
            session_id=session_id, bonded_sigma_pct=pct, bonded_amount=bonded, created_at=created_at,
            expiry=expiry, _owner=owner, _frozen=None,
        )

    def _row(self):
        f = self._frozen
        if f is not None:  # retired edge: its final state was read back when its row was freed
            return f
        return self._store.call(_st.OP_EDGE_READ, [self.edge], 3)

    def _freeze(self, active: int, released_us: int) -> None:
        self.__dict__["_frozen"] = (0, int(active), _u64(released_us))
        self.__dict__["edge"] = -1

    @property
    def is_active(self) -> bool:  # type: ignore[override]
        return bool(self._row()[1])

    @is_active.setter
    def is_active(self, v: bool) -> None:
        if not v:
            if self._frozen is None:
                self._store.call(_st.OP_RELEASE_BOND, [self.edge, _now_us()], 1)
        elif not self.is_active:
            raise ValueError("a released bond cannot be re-activated")

    @property
    def released_at(self) -> Optional[datetime]:  # type: ignore[override]
        r = self._row()
        return from_us(_i64(r[2])) if not r[1] and _i64(r[2]) >= 0 else None

    @released_at.setter
    def released_at(self, v) -> None:
        pass  # stamped by the device on release

    def __repr__(self) -> str:
        return (f"VouchRecord(vouch_id={self.vouch_id!r}, voucher_did={self.voucher_did!r}, "
                f"vouchee_did={self.vouchee_did!r}, session_id={self.session_id!r}, edge={self.edge})")


class DeviceVouchingEngine(VouchingEngine):
    """Bond edges in the device vouch table, linked per (hypervisor, session)."""

    LIST_PAGE: Optional[int] = None  # edges per listing page (default: what the bulk buffer holds)

    def __init__(self, store: GovernanceStore, tenant: int, max_exposure: Optional[float] = None) -> None:
        self._store = store
        self._tenant = tenant
        self.max_exposure = max_exposure or self.DEFAULT_MAX_EXPOSURE
        self._by_id: dict[str, DeviceVouchRecord] = {}
        self._by_edge: dict[int, DeviceVouchRecord] = {}  # edges still linked on the device
        self._order: list[DeviceVouchRecord] = []

    def __del__(self) -> None:
        try:
            edges, self._by_edge = list(self._by_edge), {}
            st, self._store = self._store, CLOSED
            st.release_tenant(self._tenant, edges)
        except Exception:
            pass

    def retire_session(self, session_id: str) -> int:
        """After a session's bonds were released (terminate), freeze each edge's
        final state into its record and return the edge rows to the store
        (OP_V_RETIRE); later vouches in the session start a new list."""
        st = self._store
        v = self._v(session_id)
        if v < 0:
            return 0
        cap = st._c.bulk_cap // 24
        r = st.call(_st.OP_V_RETIRE, [v, 0, cap], 2)
        if r[0]:
            return 0  # longer than one bulk page: the rows stay linked until the engine is dropped
        n = r[1]
        raw = st.bulk(0, 24 * n)
        edges = []
        for k in range(n):
            e, act, rel = struct.unpack_from("<qQq", raw, 24 * k)
            rec = self._by_edge.pop(e, None)
            if rec is not None:
                rec._freeze(act, rel)
            edges.append(e)
        for e in edges:  # already free on the device (V_RETIRE)
            st._c.return_row(3, e)
        return n

    def _v(self, session_id: str, create: bool = False) -> int:
        if create:
            return self._store.liability_id(self._tenant, session_id)
        return self._store.liability_lookup(self._tenant, session_id)

    def vouch_batch(self, requests: list, device: Optional[str] = None) -> list:
        """The edges already live in the device table: every request is one
        admission command to the worker (the same K05 body), queued in order."""
        out: list = []
        for r in requests:
            try:
                out.append(self.vouch(*r))
            except VouchingError as e:
                out.append(e)
        return out

    def vouch(self, voucher_did: str, vouchee_did: str, session_id: str, voucher_sigma: float,
              bond_pct: Optional[float] = None, expiry: Optional[datetime] = None) -> DeviceVouchRecord:
        st = self._store
        v = self._v(session_id, create=True)
        edge = st.alloc("E")
        now = _now()
        r = st.call(
            _st.OP_VOUCH,
            [v, st.agent_id(voucher_did), st.agent_id(vouchee_did), dbits(voucher_sigma),
             _NAN if bond_pct is None else dbits(bond_pct), to_us(expiry) if expiry is not None else -1,
             to_us(now), dbits(self.max_exposure), int(_cfg.parity_mode()), edge],
            6,
        )
        code = r[0]
        if code:  # rejected (or refused): the row was not linked and is still free on the device
            st._c.return_row(3, edge)  # RK_E
        if code == 1:
            raise VouchingError("Cannot vouch for yourself")
        if code == 2:
            raise VouchingError(
                f"Voucher σ ({voucher_sigma:.2f}) below minimum ({self.MIN_VOUCHER_SCORE:.2f})"
            )
        if code == 3:
            raise VouchingError(
                f"Circular vouching detected: {vouchee_did} already vouches for "
                f"{voucher_did} in session {session_id}"
            )
        if code == 4:
            current, bonded, limit = bitsd(r[1]), bitsd(r[2]), bitsd(r[3])
            raise VouchingError(
                f"Voucher {voucher_did} would exceed max exposure "
                f"({self.max_exposure:.0%} of σ). Current: {current:.3f}, "
                f"requested: {bonded:.3f}, limit: {limit:.3f}"
            )
        _check(r, "vouch")
        rec = DeviceVouchRecord(st, edge, _C.uuid4("vouch:"), voucher_did, vouchee_did, session_id,
                                bitsd(r[4]), bitsd(r[2]), now, expiry, owner=self)
        self._by_id[rec.vouch_id] = rec
        self._by_edge[edge] = rec
        self._order.append(rec)
        return rec

    @property
    def _vouches(self) -> dict[str, DeviceVouchRecord]:
        return dict(self._by_id)

    def compute_sigma_eff(self, vouchee_did: str, session_id: str, vouchee_sigma: float, risk_weight: float) -> float:
        v = self._v(session_id)
        r = self._store.call(
            _st.OP_SIGMA_EFF,
            [v, self._store.agent_id(vouchee_did), dbits(vouchee_sigma), dbits(risk_weight), _now_us()], 2,
        )
        return bitsd(r[1])

    def compute_sigma_eff_batch(self, requests: list) -> list[float]:
        """σ_eff for many ``(vouchee_did, session_id, vouchee_sigma, risk_weight)``
        at once: one device launch over the resident vouch lists (K03), each value
        bit-identical to :meth:`compute_sigma_eff`."""
        from agent_hypervisor_amd.ops.store_views import sigma_batch

        st = self._store
        vs = [self._v(s) for _, s, _, _ in requests]
        ag = [st.agents.lookup(d) for d, _, _, _ in requests]
        out = sigma_batch(st, vs, ag, [float(x) for _, _, x, _ in requests], [float(w) for *_, w in requests], 0)
        return [float(x) for x in out.cpu().tolist()]

    def get_total_exposure_batch(self, requests: list) -> list[float]:
        """Exposure for many ``(voucher_did, session_id)`` at once (K04 over the
        resident vouch lists; bit-identical to :meth:`get_total_exposure`)."""
        from agent_hypervisor_amd.ops.store_views import sigma_batch

        st = self._store
        out = sigma_batch(st, [self._v(s) for _, s in requests], [st.agents.lookup(d) for d, _ in requests], mode=1)
        return [float(x) for x in out.cpu().tolist()]

    def _list(self, session_id: str, flt: int, who: Optional[str]) -> list[DeviceVouchRecord]:
        """Edges of a session's device list matching ``flt`` (live by vouchee / by
        voucher / all live), in creation order; paged through the bulk buffer."""
        v = self._v(session_id)
        if v < 0:
            return []
        st = self._store
        cap = self.LIST_PAGE or st._c.bulk_cap // 64
        who_id = st.agent_id(who) if who is not None else -1
        now = _now_us()
        out: list[DeviceVouchRecord] = []
        skip = 0
        while True:
            r = st.call(_st.OP_VOUCH_LIST, [v, flt, who_id, now, 0, cap, skip], 2)
            n = r[1]
            k = min(n - skip, cap)
            raw = st.bulk(0, 64 * k)
            out.extend(self._by_edge[struct.unpack_from("<q", raw, 64 * i)[0]] for i in range(k))
            skip += k
            if skip >= n:
                return out

    def records(self, session_id: Optional[str] = None) -> list[DeviceVouchRecord]:
        if session_id is not None:  # identities are host-side; retired edges included
            return [r for r in self._order if r.session_id == session_id]
        return list(self._order)

    def get_vouchers_for(self, agent_did: str, session_id: str) -> list[DeviceVouchRecord]:
        return self._list(session_id, 1, agent_did)

    def _active_vouches_for(self, agent_did: str, session_id: str) -> list[DeviceVouchRecord]:
        return self.get_vouchers_for(agent_did, session_id)

    def get_total_exposure(self, voucher_did: str, session_id: str) -> float:
        v = self._v(session_id)
        if v < 0:
            return 0
        r = self._store.call(_st.OP_EXPOSURE, [v, self._store.agent_id(voucher_did), _now_us()], 2)
        return bitsd(r[1])

    def release_bond(self, vouch_id: str) -> None:
        rec = self._by_id.get(vouch_id)
        if rec is None:
            raise VouchingError(f"Vouch {vouch_id} not found")
        self._store.call(_st.OP_RELEASE_BOND, [rec.edge, _now_us()], 1)

    def release_session_bonds(self, session_id: str) -> int:
        v = self._v(session_id)
        if v < 0:
            return 0
        return self._store.call(_st.OP_RELEASE_SESSION, [v, _now_us()], 2)[1]

    def _creates_cycle(self, voucher_did: str, vouchee_did: str, session_id: str) -> bool:
        raise NotImplementedError("the cycle check runs inside the device vouch command (K05)")


class DeviceSlashingEngine(SlashingEngine):
    """SlashingEngine whose blacklist/clip/release/cascade runs on the device (K06)."""

    def __init__(self, vouching_engine: DeviceVouchingEngine) -> None:
        super().__init__(vouching_engine)

    def slash(self, vouchee_did: str, session_id: str, vouchee_sigma: float, risk_weight: float, reason: str,
              agent_scores: dict[str, float], cascade_depth: int = 0) -> SlashResult:
        ve: DeviceVouchingEngine = self._vouching  # type: ignore[assignment]
        st = ve._store
        v = ve._v(session_id)
        if v < 0:  # no bonds were ever posted in this session: blacklist only
            agent_scores[vouchee_did] = 0.0
            res = SlashResult(_C.uuid4("slash:"), vouchee_did, vouchee_sigma, 0.0, [], reason, session_id,
                              cascade_depth=cascade_depth)
            self._slash_history.append(res)
            return res
        pairs = [(st.agent_id(k), float(s)) for k, s in agent_scores.items()]
        raw = b"".join(struct.pack("<qd", a, s) for a, s in pairs) or b"\0" * 16
        off = st.stage(raw)
        out_cap = 1 << 16
        scores_off = 8 * out_cap
        r = st.call(
            _st.OP_SLASH,
            [v, st.agent_id(vouchee_did), dbits(vouchee_sigma), dbits(risk_weight), _now_us(), len(pairs), off,
             0, out_cap, scores_off, cascade_depth],
            3,
        )
        if r[0]:
            raise _st.StoreError(f"device slash failed with status {r[0]} (scratch/output bound)")
        words, nsc = r[1], r[2]
        stream = struct.unpack(f"<{words}Q", st.bulk(0, 8 * words))
        sc = st.bulk(scores_off, 16 * nsc)
        for k in range(nsc):
            a, s = struct.unpack_from("<qd", sc, 16 * k)
            agent_scores[st.did(a)] = s
        # rebuild SlashResults in pre-order; reasons chain "Cascade from <parent>: <reason>"
        results: list[SlashResult] = []
        reasons: dict[int, str] = {cascade_depth: reason}
        parents: dict[int, str] = {}
        i = 0
        while i < words:
            vee, depth, nclips, before = stream[i], stream[i + 1], stream[i + 2], bitsd(stream[i + 3])
            i += 4
            did = st.did(_i64(vee))
            if depth > cascade_depth:
                reasons[depth] = f"Cascade from {parents[depth - 1]}: {reasons[depth - 1]}"
            parents[depth] = did
            clips = []
            for _ in range(nclips):
                vr, b, a, e = stream[i], bitsd(stream[i + 1]), bitsd(stream[i + 2]), _i64(stream[i + 3])
                i += 4
                rec = ve._by_edge.get(e)
                clips.append(VoucherClip(st.did(_i64(vr)), b, a, risk_weight, rec.vouch_id if rec else f"edge:{e}"))
            res = SlashResult(_C.uuid4("slash:"), did, before, 0.0, clips, reasons[depth], session_id,
                              cascade_depth=int(depth))
            self._slash_history.append(res)
            results.append(res)
        return results[0]


class DeviceCommitmentEngine(CommitmentEngine):
    """Commitments of device sessions are the root/counters the terminate command wrote."""

    def __init__(self, store: GovernanceStore) -> None:
        super().__init__()
        self._store = store
        self._device: dict[str, DeviceSession] = {}
        self._batches: list = []  # batched pipelines (store_pipeline._Batch) with committed sessions

    def _record(self, sso) -> Optional[CommitmentRecord]:
        x = snapshots(self._store, [sso], parts=True)[0]
        if x.committed_at is None:
            return None
        return CommitmentRecord(
            session_id=sso.session_id, merkle_root=x.merkle_root,
            participant_dids=x.commit_dids, delta_count=x.commit_count,
            committed_at=x.committed_at,
        )

    def register(self, sso) -> None:
        """A committed device session."""
        self._device[sso.session_id] = sso

    def register_batch(self, batch) -> None:
        """The committed sessions of a batched pipeline (``batch.committed``), read
        from their rows on demand."""
        self._batches.append(batch)

    @staticmethod
    def _row(x):
        from hypervisor.core import LazyManagedSession

        return x.row if isinstance(x, LazyManagedSession) else x

    def get_commitment(self, session_id: str) -> Optional[CommitmentRecord]:
        sso = self._device.get(session_id)
        if sso is not None:
            return self._record(self._row(sso))
        for b in self._batches:
            i = b.index.get(session_id)
            if i is not None:
                return self._record(b.rowref(i)) if b.committed[i] else None
        return super().get_commitment(session_id)

    def verify(self, session_id: str, expected_root: str) -> bool:
        rec = self.get_commitment(session_id)
        return rec is not None and rec.merkle_root == expected_root

    @property
    def _commitments_view(self) -> dict[str, CommitmentRecord]:
        out = {}
        ssos = [self._row(x) for x in self._device.values()]
        snaps = snapshots(self._store, ssos, parts=True)  # one batched read per source
        for b in self._batches:
            snaps.extend(snapshots_rows(self._store, *b.rows(committed=True), parts=True))
        for x in snaps:
            if x.committed_at is not None:
                out[x.session_id] = CommitmentRecord(
                    session_id=x.session_id, merkle_root=x.merkle_root,
                    participant_dids=x.commit_dids, delta_count=x.commit_count,
                    committed_at=x.committed_at)
        out.update(self._commitments)
        return out

    @property
    def commitment_count(self) -> int:
        return len(self._commitments_view)

    def all_commitments(self) -> list[CommitmentRecord]:
        return list(self._commitments_view.values())


# ------------------------------------------------------------------ sagas


_SPECULATE = os.environ.get("AHV_STEP_SPECULATE", "1") != "0"  # A/B switch for the posted EXECUTING transition


def _transition_refused(arg, r: tuple) -> Exception:
    slot, state = arg
    return _st.StoreError(f"speculated {state.value} transition of step row {slot} refused by the device "
                          f"(from state {_STEPS[r[1]].value if r[1] < len(_STEPS) else r[1]})")


def _transition_check(slot: int, state: StepState):
    def check(r: tuple):
        if r[0] == 0:
            return None
        return _st.StoreError(f"speculated {state.value} transition of step row {slot} refused by the device "
                              f"(from state {_STEPS[r[1]].value if r[1] < len(_STEPS) else r[1]})")

    return check


class DeviceSagaStep(SagaStep):
    """Step view: FSM state, timestamps and retry counter live in the device step table."""

    def __init__(self, store: GovernanceStore, slot: int, **kw) -> None:
        self.__dict__.update(_store=store, slot=slot, execute_result=None, compensation_result=None, error=None)
        for k, v in kw.items():
            self.__dict__[k] = v

    def __del__(self) -> None:
        try:
            st = self.__dict__.get("_store")
            self.__dict__["_store"] = CLOSED
            st.release("T", self.slot)
        except Exception:
            pass

    def _row(self):
        return self._store.call(_st.OP_STEP_READ, [self.slot], 5)

    @property
    def state(self) -> StepState:  # type: ignore[override]
        return _STEPS[self._row()[1]]

    @state.setter
    def state(self, s: StepState) -> None:  # direct write outside the FSM (reference retry reset / no-undo path)
        self._store.call(_st.OP_STEP_SET, [self.slot, _STEPS.index(StepState(s)), -1], 1)
        self.__dict__["_hint"] = StepState(s)

    @property
    def retry_count(self) -> int:  # type: ignore[override]
        return self._row()[2]

    @retry_count.setter
    def retry_count(self, n: int) -> None:
        self._store.call(_st.OP_STEP_SET, [self.slot, self._row()[1], int(n)], 1)

    @property
    def started_at(self) -> Optional[datetime]:  # type: ignore[override]
        t = self._row()[3]
        return from_us(t) if t else None

    @started_at.setter
    def started_at(self, v) -> None:
        pass

    @property
    def completed_at(self) -> Optional[datetime]:  # type: ignore[override]
        t = self._row()[4]
        return from_us(t) if t else None

    @completed_at.setter
    def completed_at(self, v) -> None:
        pass

    def transition(self, new_state: StepState, retry: int = -1) -> None:
        to = _STEP_IDX[new_state] if new_state in _STEP_IDX else _STEPS.index(StepState(new_state))
        r = self._store.call(_st.OP_STEP_TRANSITION, [self.slot, to, _now_us(), retry], 2)
        self.__dict__["_hint"] = None
        self._transitioned(r, new_state)
        self.__dict__["_hint"] = _STEPS[_STEP_IDX[new_state]] if new_state in _STEP_IDX else StepState(new_state)

    async def transition_async(self, new_state: StepState, retry: int = -1) -> None:
        to = _STEP_IDX[new_state] if new_state in _STEP_IDX else _STEPS.index(StepState(new_state))
        self.__dict__["_hint"] = None
        r = await self._store.call_async(_st.OP_STEP_TRANSITION, [self.slot, to, _now_us(), retry], 2)
        self._transitioned(r, new_state)
        self.__dict__["_hint"] = _STEPS[_STEP_IDX[new_state]] if new_state in _STEP_IDX else StepState(new_state)

    def post_transition(self, new_state: StepState, retry: int = -1) -> int:
        """Post a transition without waiting (its result is read later with
        :meth:`check_posted`); the worker applies commands in order."""
        to = _STEP_IDX[new_state] if new_state in _STEP_IDX else _STEPS.index(StepState(new_state))
        self.__dict__["_hint"] = None
        return self._store.post(_st.OP_STEP_TRANSITION, [self.slot, to, _now_us(), retry], keep=True)

    async def check_posted(self, seq: int, new_state: StepState) -> None:
        self._transitioned(await self._store.result_async(seq, 2), new_state)
        self.__dict__["_hint"] = _STEPS[_STEP_IDX[new_state]] if new_state in _STEP_IDX else StepState(new_state)

    def can_speculate(self, new_state: StepState) -> bool:
        """True when this process's last known state of the step allows
        ``new_state`` (every transition of a device step goes through this object)."""
        h = self.__dict__.get("_hint")
        if not _SPECULATE or h is None:
            return False
        to = _STEPS[_STEP_IDX[new_state]] if new_state in _STEP_IDX else StepState(new_state)
        return to in STEP_TRANSITIONS.get(h, ())

    @staticmethod
    def _transitioned(r: tuple, new_state) -> None:
        if r[0]:
            frm = _STEPS[r[1]]
            allowed = STEP_TRANSITIONS.get(frm, ())
            raise SagaStateError(
                f"Invalid step transition: {frm.value} → {StepState(new_state).value}. "
                f"Allowed: {[s.value for s in allowed]}"
            )

    def __eq__(self, other) -> bool:
        return self is other

    __hash__ = object.__hash__

    def __repr__(self) -> str:
        return f"SagaStep(step_id={self.step_id!r}, action_id={self.action_id!r}, slot={self.slot})"


class DeviceSaga(Saga):
    """Saga view: FSM state and timestamps in the device saga table."""

    def __init__(self, store: GovernanceStore, slot: int, saga_id: str, session_id: str) -> None:
        self.__dict__.update(_store=store, slot=slot, saga_id=saga_id, session_id=session_id, steps=[], error=None)

    def __del__(self) -> None:
        try:
            st = self.__dict__.get("_store")
            self.__dict__["_store"] = CLOSED
            st.release("G", self.slot)
        except Exception:
            pass

    def _hdr(self):
        return self._store.call(_st.OP_SAGA_READ, [self.slot, 0, 0, 0], 5)

    @property
    def state(self) -> SagaState:  # type: ignore[override]
        return _SAGAS[self._hdr()[1]]

    @state.setter
    def state(self, s) -> None:
        raise AttributeError("saga state changes only through transition()")

    @property
    def created_at(self) -> datetime:  # type: ignore[override]
        return from_us(self._hdr()[2])

    @created_at.setter
    def created_at(self, v) -> None:
        pass

    @property
    def completed_at(self) -> Optional[datetime]:  # type: ignore[override]
        t = self._hdr()[3]
        return from_us(t) if t else None

    @completed_at.setter
    def completed_at(self, v) -> None:
        pass

    def transition(self, new_state: SagaState) -> None:
        to = _SAGAS.index(SagaState(new_state))
        r = self._store.call(_st.OP_SAGA_TRANSITION, [self.slot, to, _now_us()], 2)
        if r[0]:
            frm = _SAGAS[r[1]]
            allowed = SAGA_TRANSITIONS.get(frm, ())
            raise SagaStateError(
                f"Invalid saga transition: {frm.value} → {SagaState(new_state).value}. "
                f"Allowed: {[s.value for s in allowed]}"
            )

    def _step_states(self) -> list[StepState]:
        n, off, inl = self._store.index_args([s.slot for s in self.steps])
        self._store.call(_st.OP_SAGA_READ, [self.slot, n, off, 0], 1, inl)
        raw = self._store.bulk(0, 32 * n)
        return [_STEPS[struct.unpack_from("<Q", raw, 32 * k)[0] & 0xFF] for k in range(n)]

    @property
    def committed_steps(self) -> list[SagaStep]:
        return [s for s, stt in zip(self.steps, self._step_states()) if stt is StepState.COMMITTED]

    @property
    def committed_steps_reversed(self) -> list[SagaStep]:
        """K14 on the device: committed steps in reverse order."""
        n, off, inl = self._store.index_args([s.slot for s in self.steps])
        r = self._store.call(_st.OP_SAGA_PLAN, [self.slot, n, off, 0], 6, inl)
        m = r[5]
        raw = self._store.bulk(0, 8 * m)
        return [self.steps[struct.unpack_from("<Q", raw, 8 * k)[0]] for k in range(m)]

    def __eq__(self, other) -> bool:
        return self is other

    __hash__ = object.__hash__

    def __repr__(self) -> str:
        return f"Saga(saga_id={self.saga_id!r}, session_id={self.session_id!r}, slot={self.slot})"


class DeviceSagaOrchestrator(SagaOrchestrator):
    """SagaOrchestrator with the step/saga FSM (K13) and compensation plan (K14) on the device.

    Executors and compensators are user coroutines and stay on the host event
    loop; every state change they cause is a device command.
    """

    def __init__(self, store: GovernanceStore, owner: Optional[DeviceSession] = None, reg=None) -> None:
        self._store = store
        self._sagas: dict[str, DeviceSaga] = {}
        self._owner = owner  # the session whose speculated step transitions these are
        self._reg = reg  # the hypervisor's saga-row registry (SessionTable.saga_rows), when known

    def _guard(self) -> None:
        o = self._owner
        if o is not None:
            o._guard()

    async def execute_sagas(self, saga_ids, executors, compensator=None, compensate: bool = True,
                            device: Optional[str] = None) -> list:
        """The sagas' state machines already live in the store's rows: every step
        runs through the store worker's FSM (``device`` is accepted for API
        symmetry — there is no separate batch engine to replay into)."""
        return await SagaOrchestrator.execute_sagas(self, saga_ids, executors, compensator, compensate, None)

    def create_saga(self, session_id: str, saga_id: Optional[str] = None) -> DeviceSaga:
        slot = self._store.alloc("G")
        saga = DeviceSaga(self._store, slot, saga_id or _C.uuid4("saga:"), session_id)
        self._store.post(_st.OP_SAGA_CREATE, [slot, _now_us()])
        self._sagas[saga.saga_id] = saga
        reg = self._reg
        if reg is not None:
            reg.append(slot)
        return saga

    def add_step(self, saga_id: str, action_id: str, agent_did: str, execute_api: str,
                 undo_api: Optional[str] = None, timeout_seconds: int = 300, max_retries: int = 0) -> DeviceSagaStep:
        saga = self._get_saga(saga_id)
        slot = self._store.alloc("T")
        step = DeviceSagaStep(
            self._store, slot, step_id=_C.uuid4("step:"), action_id=action_id, agent_did=agent_did,
            execute_api=execute_api, undo_api=undo_api, timeout_seconds=timeout_seconds, max_retries=max_retries,
        )
        self._store.post(_st.OP_STEP_ADD, [saga.slot, slot, int(bool(undo_api)), int(max_retries)])
        step.__dict__["_hint"] = StepState.PENDING
        saga.steps.append(step)
        return step

    async def execute_step(self, saga_id: str, step_id: str, executor: Callable[..., Any]) -> Any:
        if _CTL:
            _C.ctl_guard(self._owner)
        else:
            self._guard()
        saga = self._get_saga(saga_id)
        step = self._get_step(saga, step_id)
        attempts = 1 + step.max_retries
        last: Optional[Exception] = None
        for attempt in range(attempts):
            # the EXECUTING transition is posted and the executor starts at once when this
            # process knows the step's state allows it (its result is checked right after)
            if _CTL and _SPECULATE and type(step) is DeviceSagaStep:
                seq = _C.ctl_step_begin(step, attempt)
            else:
                seq = step.post_transition(StepState.EXECUTING, retry=attempt) \
                    if step.can_speculate(StepState.EXECUTING) else None
            if seq is None:
                await step.transition_async(StepState.EXECUTING, retry=attempt)
            try:
                result = await await_with_timeout(executor(), step.timeout_seconds)
            except asyncio.CancelledError:
                if seq is not None:  # the posted transition's kept result will never be read
                    self._store.discard(seq)
                raise
            except asyncio.TimeoutError:
                last = SagaTimeoutError(
                    f"Step {step_id} timed out after {step.timeout_seconds}s "
                    f"(attempt {attempt + 1}/{attempts})"
                )
            except Exception as e:  # executor failure
                last = e
            else:
                step.execute_result = result
                if seq is not None and _SPEC_LIFECYCLE:
                    # EXECUTING was known-valid when posted, and COMMITTED is allowed from
                    # EXECUTING: neither needs the device's answer before returning —
                    # both are verified with the store's next interaction
                    if _CTL and type(step) is DeviceSagaStep:
                        _C.ctl_step_commit(self._owner, step, seq)
                        return result
                    st = self._store
                    slot = step.slot
                    st.expect(seq, _OK, (self._owner, _transition_refused, (slot, StepState.EXECUTING)))
                    st._c.post_expect(_st.OP_STEP_TRANSITION, [slot, _COMMITTED_IDX, _now_us(), -1], None, _OK,
                                      (self._owner, _transition_refused, (slot, StepState.COMMITTED)))
                    step.__dict__["_hint"] = StepState.COMMITTED
                    return result
                if seq is not None:
                    await step.check_posted(seq, StepState.EXECUTING)
                await step.transition_async(StepState.COMMITTED)
                return result
            if seq is not None:
                await step.check_posted(seq, StepState.EXECUTING)
            step.error = str(last)
            step.transition(StepState.FAILED)
            if attempt < attempts - 1:
                step.state = StepState.PENDING
                step.error = None
                await asyncio.sleep(self.DEFAULT_RETRY_DELAY_SECONDS * (attempt + 1))
        if last is not None:
            raise last
        raise SagaStateError("Step execution failed with no error captured")

    async def compensate(self, saga_id: str, compensator: Callable[[SagaStep], Any]) -> list[SagaStep]:
        self._guard()
        saga = self._get_saga(saga_id)
        saga.transition(SagaState.COMPENSATING)
        failed: list[SagaStep] = []
        for step in saga.committed_steps_reversed:
            if not step.undo_api:
                step.state = StepState.COMPENSATION_FAILED
                step.error = "No Undo_API available"
                failed.append(step)
                continue
            step.transition(StepState.COMPENSATING)
            try:
                res = await await_with_timeout(compensator(step), step.timeout_seconds)
            except asyncio.TimeoutError:
                step.error = f"Compensation timed out after {step.timeout_seconds}s"
            except Exception as e:
                step.error = f"Compensation failed: {e}"
            else:
                step.compensation_result = res
                step.transition(StepState.COMPENSATED)
                continue
            step.transition(StepState.COMPENSATION_FAILED)
            failed.append(step)
        if failed:
            saga.transition(SagaState.ESCALATED)
            saga.error = f"{len(failed)} step(s) failed compensation — Joint Liability slashing triggered"
        else:
            saga.transition(SagaState.COMPLETED)
        return failed


def snapshots(store: GovernanceStore, ssos: list, parts: bool = False) -> list[SessionSnapshot]:
    """Snapshots of many device sessions with O(1) store commands (OP_SESS_READ_MANY)."""
    if not ssos:
        return []
    return snapshots_rows(store, [x.slot for x in ssos], [x.session_id for x in ssos],
                          [x.creator_did for x in ssos], parts)


def snapshots_rows(store: GovernanceStore, slots, ids: list, creators: list,
                   parts: bool = False) -> list[SessionSnapshot]:
    """:func:`snapshots` from row arrays (slot, session id, creator DID per row)."""
    if not len(ids):
        return []
    hdr, prt = store.read_sessions(slots, parts=parts)
    out = []
    for i, sid in enumerate(ids):
        h = hdr[i]
        s = SessionSnapshot()
        w0 = int(h[0])
        s.session_id = sid
        s.state = _STATES[w0 & 0xFF]
        s.consistency_mode = _MODES[(w0 >> 8) & 0xFF]
        w1 = int(h[1])
        pc = w1 & 0xFFFFFFFF
        s.participant_count = (w1 >> 32) & 0xFFFFFFFF
        s.created_at = from_us(_i64(int(h[2])))
        te = _i64(int(h[3]))
        s.terminated_at = from_us(te) if te else None
        s.delta_count = int(h[4]) & 0xFFFFFFFF
        s.creator_did = creators[i]
        c = _i64(int(h[7]))
        s.committed_at = from_us(c) if c else None
        s.commit_count = (int(h[4]) >> 32) & 0xFFFFFFFF
        s.merkle_root = "".join(f"{int(w):016x}" for w in h[12:16]) if c else None
        if parts:
            plist, committed = [], []
            for k in range(pc):
                a, fl, sr, se, j = (int(x) for x in prt[i, k])
                if (fl >> 9) & 1:  # P_COMMITTED: active when the root was committed
                    committed.append(store.did(_i64(a)))
                if (fl >> 8) & 1:  # P_ACTIVE
                    plist.append(SessionParticipant(
                        agent_did=store.did(_i64(a)), ring=_RINGS[fl & 0xFF], sigma_raw=bitsd(sr), sigma_eff=bitsd(se),
                        joined_at=from_us(_i64(j)), is_active=True))
            s.participants = plist
            s.commit_dids = committed
        else:
            s.participants = s.commit_dids = None
        out.append(s)
    return out


def saga_rows(store: GovernanceStore, sagas: list) -> dict:
    """States / timestamps of many device sagas and their steps: one column gather
    per field (O(1) store commands).  ``{"g_state": [...], "steps": {col: [...]}}``
    in saga order, steps flattened in saga-then-step order."""
    gi = [g.slot for g in sagas]
    ti = [st.slot for g in sagas for st in g.steps]
    out = store.gather({"g_state": gi, "g_created": gi, "g_completed": gi,
                        "t_state": ti, "t_retry": ti, "t_started": ti, "t_completed": ti})
    return out


class _ClosedStore:
    """Stands in for the store in the views of a closed hypervisor: their rows were
    returned by :func:`close_hypervisor`, so any use raises (a freed row may already
    hold another session) and a late finaliser releases nothing twice."""

    __slots__ = ()

    def release(self, kind, row) -> None:
        pass

    def release_many(self, kind, rows) -> None:
        pass

    def release_tenant(self, tenant, edges) -> None:
        pass

    def __getattr__(self, name):
        raise _st.StoreError("this session belongs to a closed Hypervisor: its store rows were released")

    def __bool__(self) -> bool:
        return True


CLOSED = _ClosedStore()


def _close_views(st: GovernanceStore, m, acc: Optional[tuple] = None) -> None:
    """Release the rows of one built device session and detach its views.  Each
    view is handled on its own: in cyclic garbage some of them may already have
    run their finaliser (which detached them after releasing their row).
    ``acc``: (session, delta, saga, step) row lists the caller releases in one
    native call per table instead."""
    own = acc is None
    if own:
        acc = ([], [], [], [])
    s_rows, d_rows, g_rows, t_rows = acc
    sso, de, orch = m.sso, m.delta_engine, m.saga
    if getattr(sso, "_store", None) is st:
        s_rows.append(sso.slot)
        sso._store = CLOSED
    if type(de) is DeviceDeltaEngine or isinstance(de, DeviceDeltaEngine):
        if de._store is st:
            rows, de._rows = de._rows, []
            d_rows.extend(rows)
            de._store = CLOSED
        for d in de._deltas:
            d.__dict__["_store"] = CLOSED
    if type(orch) is DeviceSagaOrchestrator or isinstance(orch, DeviceSagaOrchestrator):
        for g in orch._sagas.values():
            gd = g.__dict__
            if gd.get("_store") is st:
                g_rows.append(g.slot)
                gd["_store"] = CLOSED
            for x in g.steps:
                xd = x.__dict__
                if xd.get("_store") is st:
                    t_rows.append(x.slot)
                    xd["_store"] = CLOSED
        orch._store = CLOSED
    if own:
        _release_acc(st, acc)


def _release_acc(st: GovernanceStore, acc: tuple) -> None:
    for kind, rows in zip("SDGT", acc):
        if rows:
            st.release_many(kind, rows)


def close_hypervisor(hv) -> int:
    """Return every store row a device-backed hypervisor holds — sessions, their
    participants' rows, delta chains with their arena records, sagas, steps, vouch
    edges and liability-session rows — to the store, whatever Python still refers
    to them; afterwards its views raise :class:`StoreError`.  Returns the number
    of sessions closed.  Called by :meth:`Hypervisor.close` (and when the
    hypervisor object goes away)."""
    st = hv._store
    if st is None or st is CLOSED or getattr(st, "_closed", False):
        return 0
    if _CTL:
        n = _C.ctl_close_hypervisor(hv)  # one native pass (own sessions, no vouching engine)
        if n >= 0:
            return n
    # No wait for the commands still in flight: the worker runs commands in order, so
    # the FREE_ROWS that later reclaims these rows executes after every command posted
    # for them (a divergence of a speculated post goes to its session, now closed).
    n = 0
    acc = ([], [], [], [])
    own = hv._sessions._own
    for seg in list(hv._sessions._segs):  # every segment, including emptied batches (their dead rows)
        if isinstance(seg, list):
            for sid in seg:
                m = own.get(sid)
                if m is not None:
                    _close_views(st, m, acc)
                    n += 1
            continue
        for m in list(seg.views.values()):
            _close_views(st, m, acc)
        seg.release(np.arange(len(seg.slots), dtype=np.int64))
        n += len(seg.index)
    _release_acc(st, acc)
    ve = hv.__dict__.get("vouching")  # engines never used were never built (Hypervisor.__getattr__)
    if isinstance(ve, DeviceVouchingEngine) and ve._store is st:
        st.release_tenant(ve._tenant, list(ve._by_edge))
        for rec in ve._by_edge.values():
            rec.__dict__["_store"] = CLOSED
        ve._by_edge = {}
        ve._store = CLOSED
    elif ve is None:
        st.release_tenant(hv._tenant, [])
    cm = hv.__dict__.get("commitment")
    if isinstance(cm, DeviceCommitmentEngine):
        cm._store = CLOSED
    hv._store = CLOSED
    return n


def session_views(store: GovernanceStore, sso: DeviceSession, saga_reg=None):
    """(delta engine, saga orchestrator) for a device session (``saga_reg``: the
    hypervisor's saga-row registry the orchestrator appends to)."""
    return DeviceDeltaEngine(store, sso.slot, sso.session_id, sso), DeviceSagaOrchestrator(store, sso, saga_reg)


_S_ARCHIVED, _S_TERMINATING = _STATES.index(SessionState.ARCHIVED), _STATES.index(SessionState.TERMINATING)
_G_LIVE = (_SAGAS.index(SagaState.RUNNING), _SAGAS.index(SagaState.COMPENSATING))


def counters(hv) -> dict:
    """The REST ``/stats`` counters of a device-backed hypervisor, reduced on the
    device over its rows: sessions (table size), active sessions (row state not
    archived / terminating), participants (Σ active participant rows), active
    sagas (RUNNING or COMPENSATING) and sagas, vouches (the engine's records).
    O(1) store commands (one release of the worker's writes) and one 4-word copy
    back, however many sessions (reference api/server.py:144-163)."""
    import torch

    st = hv._store
    tab = hv._sessions
    slots = tab.session_slots()
    g_own = np.frombuffer(tab.saga_rows, dtype=np.int64) if len(tab.saga_rows) else np.zeros(0, np.int64)
    grows = np.concatenate([g_own, tab.batch_saga_rows()])
    out = {"total_sessions": len(tab), "total_vouches": len(hv.vouching.records()), "total_sagas": int(len(grows))}
    if not len(slots) and not len(grows):
        out.update(active_sessions=0, total_participants=0, active_sagas=0)
        return out
    st.drain()
    if st.device.type == "cuda":
        st.flush()
    dev = st.device
    t = st.tables
    res = torch.zeros(3, dtype=torch.int64, device=dev)
    if len(slots):
        ix = torch.from_numpy(slots).to(dev)
        sst = t["s_state"].index_select(0, ix)
        res[0] = ((sst != _S_ARCHIVED) & (sst != _S_TERMINATING)).sum()
        res[1] = t["s_pactive"].index_select(0, ix).to(torch.int64).sum()
    if len(grows):
        gs = t["g_state"].index_select(0, torch.from_numpy(grows).to(dev))
        res[2] = ((gs == _G_LIVE[0]) | (gs == _G_LIVE[1])).sum()
    a, p, g = res.cpu().tolist()
    out.update(active_sessions=int(a), total_participants=int(p), active_sagas=int(g))
    return out


# ------------------------------------------------------------------ native control plane

# The per-call hot paths in C++ (csrc/host/py_control.cpp): the same objects and
# semantics, without a Python frame per command (AHV_NATIVE_CTL=0: the Python path).
_CTL = os.environ.get("AHV_NATIVE_CTL", "1") != "0" and hasattr(_C, "ctl_init")


def _install_native() -> None:
    from hypervisor import _clock

    DeviceDeltaEngine._py_capture = DeviceDeltaEngine.__dict__["capture"]
    DeviceSagaOrchestrator._py_create_saga = DeviceSagaOrchestrator.__dict__["create_saga"]
    DeviceSagaOrchestrator._py_add_step = DeviceSagaOrchestrator.__dict__["add_step"]
    _C.ctl_init({
        "GovernanceStore": GovernanceStore, "DeviceSession": DeviceSession, "DeviceDelta": DeviceDelta,
        "DeviceDeltaEngine": DeviceDeltaEngine, "DeviceSagaOrchestrator": DeviceSagaOrchestrator,
        "DeviceSaga": DeviceSaga, "DeviceSagaStep": DeviceSagaStep, "DeviceCommitmentEngine": DeviceCommitmentEngine,
        "CLOSED": CLOSED, "clock_dict": _clock.__dict__, "now": _clock.now, "to_us": _clock.to_us,
        "mode_eventual": ConsistencyMode.EVENTUAL, "mode_strong": ConsistencyMode.STRONG,
        "step_pending": StepState.PENDING, "step_executing": StepState.EXECUTING,
        "step_committed": StepState.COMMITTED,
        "exec_from": frozenset(s for s in StepState if StepState.EXECUTING in STEP_TRANSITIONS.get(s, ())),
        "err_create": _create_refused, "err_join": _join_diverged, "err_activate": _activate_refused,
        "err_transition": _transition_refused, "fb_capture": DeviceDeltaEngine._py_capture,
        "fb_create_saga": DeviceSagaOrchestrator._py_create_saga, "fb_add_step": DeviceSagaOrchestrator._py_add_step,
        "s_handshaking": _S_HANDSHAKING, "s_active": _S_ACTIVE, "step_executing_idx": _STEP_IDX[StepState.EXECUTING],
        "step_committed_idx": _COMMITTED_IDX, "spec_lifecycle": _SPEC_LIFECYCLE, "step_speculate": _SPECULATE,
        "spec_terminate": _SPEC_TERMINATE, "check_terminate": _CHECK_TERMINATE,
        "close_hv_fast": _C.ctl_close_hypervisor,
    })
    # finalisers: a view the hypervisor's close detached costs one native call
    vdel = _C.ctl_method(_C.ctl_view_del)
    for cls in (DeviceSession, DeviceDeltaEngine, DeviceSaga, DeviceSagaStep):
        cls._py_del = cls.__dict__["__del__"]
        cls.__del__ = vdel
    from hypervisor.core import Hypervisor

    Hypervisor._py_del = Hypervisor.__dict__["__del__"]
    Hypervisor.__del__ = _C.ctl_method(_C.ctl_hv_del)
    DeviceDeltaEngine.capture = _C.ctl_method(_C.ctl_capture)
    DeviceSagaOrchestrator.create_saga = _C.ctl_method(_C.ctl_create_saga)
    DeviceSagaOrchestrator.add_step = _C.ctl_method(_C.ctl_add_step)


if _CTL:
    _install_native()


__all__ = [
    "DeviceSession", "DeviceDelta", "DeviceDeltaEngine", "DeviceVouchRecord", "DeviceVouchingEngine",
    "DeviceSlashingEngine", "DeviceCommitmentEngine", "DeviceSaga", "DeviceSagaStep", "DeviceSagaOrchestrator",
    "SessionSnapshot", "snapshots", "saga_rows",
]
