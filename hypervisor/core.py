"""Hypervisor: the top-level orchestrator of shared multi-agent sessions.

Parity target: reference ``core.py:37-298``.

Shared engines: vouching, slashing, ring enforcer, action classifier, history
verifier, commitment, GC.  Per session (:class:`ManagedSession`): the SSO (with
its VFS), a reversibility registry, a delta engine and a saga orchestrator.

``join_session`` (the admission "forward pass"):

1. IATP manifest enrichment when an adapter and manifest are given (manifest
   actions fill in missing ``actions``; the σ hint replaces ``sigma_raw == 0.0``);
2. register actions; any irreversible action forces STRONG consistency;
3. history verification (an untrustworthy history forces Ring 3);
4. σ resolution — Nexus when ``sigma_raw == 0.0``; with an explicit σ *and* a
   history, the lower of the two;
5. ring = ``compute_ring(σ)``; ``sso.join``.

``terminate_session``: TERMINATING → Merkle root → commitment → release the
session's bonds → GC → ARCHIVED; returns the root (``None`` with audit off or no
deltas).

``verify_behavior``: CMVK drift check; HIGH/CRITICAL drift slashes the agent
(ω = 0.95) against a snapshot of participant σ and reports to Nexus.  As in the
reference the participant's own σ/ring are left unchanged unless
``demote_on_slash=True`` (Q06).

Additions: an optional ``event_bus`` that receives lifecycle events (the
reference never emitted, Q03); an optional ``declared_history`` for join (Q23);
and :meth:`Hypervisor.pipeline_batch` / :meth:`Hypervisor.run_pipelines`, which
run the pipeline for thousands of sessions in one device launch over the same
store rows the per-call API uses (one device state).

Device-authoritative mode (``Hypervisor(device="cuda")``, the default when a HIP
device is visible; ``AHV_STORE``): sessions, participants, the audit chain,
vouch bonds, sagas and commitments live in the gfx950 state store
(:mod:`agent_hypervisor_amd.models.store`) and every call below is a command to
its resident worker (:mod:`hypervisor._device`) — the join ring gate (K01),
capture hashing (K08), the terminate pipeline (K09 root → commit → K07 bond
release → GC → archive) and the slash cascade (K06) all run on the device.
``device="cpu"`` runs the same command processor on the host (twin for tests);
``device="host"`` keeps the pure host engines.
"""

from __future__ import annotations

import logging
from typing import Any, Optional

from hypervisor.audit.commitment import CommitmentEngine
from hypervisor.config import store_mode as _store_mode
from hypervisor.audit.delta import DeltaEngine
from hypervisor.audit.gc import EphemeralGC, RetentionPolicy
from hypervisor.liability.slashing import SlashingEngine
from hypervisor.liability.vouching import VouchingEngine
from hypervisor.models import ActionDescriptor, ConsistencyMode, ExecutionRing, SessionConfig, SessionState
from hypervisor.reversibility.registry import ReversibilityRegistry
from hypervisor.rings.classifier import ActionClassifier
from hypervisor.rings.enforcer import RingEnforcer
from hypervisor.saga.orchestrator import SagaOrchestrator
from hypervisor.session import SharedSessionObject
from hypervisor.session.table import SessionTable
from hypervisor.verification.history import TransactionHistoryVerifier

logger = logging.getLogger(__name__)

_STRONG = ConsistencyMode.STRONG


class ManagedSession:
    """A session plus the engines scoped to it."""

    __slots__ = ("sso", "reversibility", "delta_engine", "saga")

    def __init__(self, sso: SharedSessionObject, delta_engine=None, saga=None) -> None:
        self.sso = sso
        sid = sso.session_id
        self.reversibility = ReversibilityRegistry(sid)
        self.delta_engine = delta_engine if delta_engine is not None else DeltaEngine(sid)
        self.saga = saga if saga is not None else SagaOrchestrator()


class LazyManagedSession(ManagedSession):
    """Transient stand-in for a session a batched pipeline wrote into the device
    store (:meth:`Hypervisor.run_pipelines`) whose Python views are not built yet:
    :meth:`SessionTable.values` yields one per such session.  ``row`` identifies
    the session row without building anything; any other attribute builds the
    views (kept by the batch) and reads through."""

    __slots__ = ("_batch", "_index")

    def __init__(self, batch, index: int) -> None:  # noqa: D107 - views come later
        self._batch = batch
        self._index = index

    @property
    def row(self):
        """Identity of the session row (slot, id, creator) without building views."""
        return self._batch.rowref(self._index)

    def __getattr__(self, name):
        if name.startswith("_"):
            raise AttributeError(name)
        return getattr(self._batch.view(self._index), name)


_DEVICE_MOD = None


def _device_mod():
    """``hypervisor._device`` (imported on first use: host-only processes never load
    torch or the device store)."""
    global _DEVICE_MOD
    if _DEVICE_MOD is None:
        from hypervisor import _device

        _DEVICE_MOD = _device
    return _DEVICE_MOD


class Hypervisor:
    def __init__(
        self,
        retention_policy: Optional[RetentionPolicy] = None,
        max_exposure: Optional[float] = None,
        nexus: Optional[Any] = None,
        cmvk: Optional[Any] = None,
        iatp: Optional[Any] = None,
        event_bus: Optional[Any] = None,
        demote_on_slash: bool = False,
        device: Optional[str] = None,
        store: Optional[Any] = None,
    ) -> None:
        mode = _store_mode(device) if store is None else str(store.device)
        self._store = None
        if mode == "host":
            self.vouching = VouchingEngine(max_exposure=max_exposure)
            self.slashing = SlashingEngine(self.vouching)
            self.commitment = CommitmentEngine()
        else:
            _device = _device_mod()
            self._store = store if store is not None else _device._shared_store(mode)
            self._tenant = self._store.new_tenant()
            # the device vouching / slashing / commitment engines are built on first
            # use (__getattr__): a hypervisor that runs a few pipelines and closes
            # never pays for the ones it does not touch
            self._max_exposure = max_exposure
        self.device = mode
        if mode == "host":
            self.ring_enforcer = RingEnforcer()
            self.classifier = ActionClassifier()
        # (device-backed: the ring gate runs on the device; ring_enforcer / classifier
        # are built on first use, see __getattr__)
        self.verifier = TransactionHistoryVerifier()
        self.gc = EphemeralGC(retention_policy)
        self.nexus = nexus
        self.cmvk = cmvk
        self.iatp = iatp
        self.event_bus = event_bus
        self.demote_on_slash = demote_on_slash
        self._sessions = SessionTable()
        self.batched_sessions = 0  # sessions written by pipeline_batch / run_pipelines (ordinary sessions)

    _LAZY_ENGINES = frozenset(("vouching", "slashing", "commitment"))

    def __getattr__(self, name: str):
        # only reached for attributes not set yet: the device engines of a
        # device-backed hypervisor, built together on first use
        d = self.__dict__
        if name == "ring_enforcer" or name == "classifier":
            d["ring_enforcer"] = RingEnforcer()
            d["classifier"] = ActionClassifier()
            return d[name]
        if name in Hypervisor._LAZY_ENGINES and d.get("_store") is not None:
            _device = _device_mod()
            st = d["_store"]
            if name == "commitment":  # every terminate registers here; no vouching engine needed
                cm = d["commitment"] = _device.DeviceCommitmentEngine(st)
                pend = d.pop("_commits", None)  # sessions terminates committed before it existed
                if pend:
                    cm._device.update(pend)
                return d[name]
            ve = d["vouching"] = _device.DeviceVouchingEngine(st, d["_tenant"], d.get("_max_exposure"))
            d["slashing"] = _device.DeviceSlashingEngine(ve)
            if "commitment" not in d:
                self.__getattr__("commitment")
            return d[name]
        raise AttributeError(f"{type(self).__name__!r} object has no attribute {name!r}")

    # -- lifetime ------------------------------------------------------------
    def close(self) -> int:
        """Device-backed: return every store row this hypervisor holds (sessions,
        participants, delta chains and their records, sagas, steps, vouch edges)
        to the shared store now, whatever Python still refers to them; its session
        views raise afterwards.  Also runs when the hypervisor object is dropped, so
        row lifetime follows the hypervisor, not the collector.  Returns the number
        of sessions closed (0 for host engines, which hold no device rows)."""
        if self._store is None:
            return 0
        return _device_mod().close_hypervisor(self)

    def __del__(self) -> None:
        try:
            if getattr(self, "_store", None) is not None:
                self.close()
        except Exception:  # noqa: BLE001 - interpreter shutdown / store already closed
            pass

    def __enter__(self) -> "Hypervisor":
        return self

    def __exit__(self, *exc) -> None:
        self.close()

    async def __aenter__(self) -> "Hypervisor":
        return self

    async def __aexit__(self, *exc) -> None:
        self.close()

    # -- events --------------------------------------------------------------
    def _emit(self, etype, session_id=None, agent_did=None, **payload) -> None:
        bus = self.event_bus
        if bus is not None:
            from hypervisor.observability.event_bus import HypervisorEvent

            bus.emit(HypervisorEvent(event_type=etype, session_id=session_id, agent_did=agent_did, payload=payload))

    # -- lifecycle -------------------------------------------------------------
    async def create_session(self, config: SessionConfig, creator_did: str,
                             session_id: Optional[str] = None) -> ManagedSession:
        """``session_id``: an explicit id (extension: the sharded façade mints ids
        that route to the owner rank); default ``session:{uuid4}``."""
        if session_id is not None and session_id in self._sessions:
            raise ValueError(f"Session {session_id} already exists")
        if self._store is not None:
            _device = _device_mod()
            views = _device._C.ctl_session(self._store, config, creator_did, session_id, self._sessions.saga_rows) \
                if _device._CTL and _device._SPEC_LIFECYCLE else None  # native: row + views in one call
            if views is None:
                sso = _device.DeviceSession(self._store, config, creator_did, session_id=session_id)  # HANDSHAKING
                views = (sso, *_device.session_views(self._store, sso, self._sessions.saga_rows))
            managed = ManagedSession(*views)
            sso = views[0]
        else:
            sso = SharedSessionObject(config=config, creator_did=creator_did, session_id=session_id)
            sso.begin_handshake()
            managed = ManagedSession(sso)
        self._sessions[sso.session_id] = managed
        if self.event_bus is not None:
            from hypervisor.observability.event_bus import EventType

            self._emit(EventType.SESSION_CREATED, sso.session_id, creator_did)
        return managed

    async def join_session(
        self,
        session_id: str,
        agent_did: str,
        actions: Optional[list[ActionDescriptor]] = None,
        sigma_raw: float = 0.0,
        manifest: Optional[Any] = None,
        agent_history: Optional[Any] = None,
        declared_history: Optional[list] = None,
    ) -> ExecutionRing:
        managed = self._get_session(session_id)
        if self.iatp and manifest:
            analysis = (
                self.iatp.analyze_manifest_dict(manifest)
                if isinstance(manifest, dict)
                else self.iatp.analyze_manifest(manifest)
            )
            if not actions:
                actions = analysis.actions
            if sigma_raw == 0.0:
                sigma_raw = analysis.sigma_hint
            logger.debug("IATP manifest parsed for %s: ring_hint=%s", agent_did, analysis.ring_hint)
        if actions:
            managed.reversibility.register_from_manifest(actions)
        if managed.reversibility.has_non_reversible_actions():
            managed.sso.force_consistency_mode(_STRONG)

        verification = self.verifier.verify(agent_did, declared_history)

        sigma_eff = sigma_raw
        if self.nexus:
            if sigma_raw == 0.0:
                sigma_eff = self.nexus.resolve_sigma(agent_did, history=agent_history)
                logger.debug("Nexus resolved sigma=%.3f for %s", sigma_eff, agent_did)
            elif agent_history:
                sigma_eff = min(sigma_raw, self.nexus.resolve_sigma(agent_did, history=agent_history))

        if self._store is not None:  # ring gate (K01) + admission on the device
            _d = _device_mod()
            got = _d._C.ctl_join(managed.sso, agent_did, sigma_raw, sigma_eff, verification.is_trustworthy) \
                if _d._CTL else None  # a join the device will admit: posted, verified later
            if got is not None:
                ring = _d._RINGS[got]
            else:
                ring = await managed.sso.join_gated_async(agent_did, sigma_raw, sigma_eff,
                                                          verification.is_trustworthy)
        else:
            ring = self.ring_enforcer.compute_ring(sigma_eff)
            if not verification.is_trustworthy:
                ring = ExecutionRing.RING_3_SANDBOX
            managed.sso.join(agent_did=agent_did, sigma_raw=sigma_raw, sigma_eff=sigma_eff, ring=ring)
        if self.event_bus is not None:
            from hypervisor.observability.event_bus import EventType

            self._emit(EventType.SESSION_JOINED, session_id, agent_did, sigma_eff=sigma_eff)
            self._emit(EventType.RING_ASSIGNED, session_id, agent_did, ring=int(ring.value))
        return ring

    async def activate_session(self, session_id: str) -> None:
        sso = self._get_session(session_id).sso
        if self._store is not None:
            _d = _device_mod()
            if not (_d._CTL and _d._C.ctl_activate(sso)):  # native: a known-good activation is posted
                await sso.activate_async()
        else:
            sso.activate()
        if self.event_bus is not None:
            from hypervisor.observability.event_bus import EventType

            self._emit(EventType.SESSION_ACTIVATED, session_id)

    async def terminate_session(self, session_id: str) -> Optional[str]:
        managed = self._get_session(session_id)
        if self._store is not None:
            return await self._terminate_device(session_id, managed)
        sso = managed.sso
        sso.terminate()
        de = managed.delta_engine
        root = None
        if sso.config.enable_audit:
            root = de.compute_merkle_root()
            if root:
                self.commitment.commit(
                    session_id=session_id,
                    merkle_root=root,
                    participant_dids=[p.agent_did for p in sso.participants],
                    delta_count=de.turn_count,
                )
        self.vouching.release_session_bonds(session_id)
        self.gc.collect(session_id=session_id, vfs=sso.vfs, delta_engine=de, delta_count=de.turn_count)
        sso.archive()
        if self.event_bus is not None:
            from hypervisor.observability.event_bus import EventType

            self._emit(EventType.SESSION_TERMINATED, session_id, merkle_root=root)
            if root:
                self._emit(EventType.AUDIT_COMMITTED, session_id, merkle_root=root)
            self._emit(EventType.AUDIT_GC_COLLECTED, session_id)
            self._emit(EventType.SESSION_ARCHIVED, session_id)
        return root

    async def _terminate_device(self, session_id: str, managed: ManagedSession) -> Optional[str]:
        """One device command: terminate → Merkle root (K09) → commit → release the
        session's bonds (K07) → GC retention count → archive."""
        _d = _device_mod()
        sso, de, st = managed.sso, managed.delta_engine, self._store
        pre = _d._C.ctl_close(self, session_id, sso, de) \
            if _d._CTL and _d._CHECK_TERMINATE and not _d._SPEC_TERMINATE else None
        if pre is not None:
            # native: guard, GC cutoff, the host's root / GC-count prediction and the
            # posted close in one call; the bookkeeping that needs no device answer
            # runs while the hash engine finishes, then the root is awaited
            seq, root_pred, expired_pred, n = pre
            self._terminate_gc(session_id, sso, de, expired_pred, n)
            r = await st.result_async(seq, 13, 0)
            return _d._C.ctl_close_finish(self, session_id, sso, r, (root_pred, expired_pred))
        guard = getattr(sso, "_guard", None)
        if guard is not None:  # a speculation of this session the device refused raises here
            guard()
        now_us = _d._now_us()
        v = st.liability_lookup(self._tenant, session_id)
        cutoff = now_us - int(self.gc.policy.delta_retention_days * 86_400_000_000)
        n, off, inl = st.index_args(de._indices())
        audit = bool(sso.config.enable_audit)
        args = [sso.slot, n, off, now_us, v, cutoff, int(audit)]
        spec = _d.close_prediction(sso, de, v, audit, cutoff) if guard is not None else None
        # awaited: the device's root is returned, checked against the host's prediction
        check = _d.close_prediction(sso, de, v, audit, cutoff, check=True) \
            if spec is None and guard is not None and _d._CHECK_TERMINATE else None
        sso._m_forget()  # the row leaves the mirrored states (terminate → archive)
        if spec is not None:
            # the host knows the outcome (root from its digest predictions): post the
            # close without waiting for the hash engine; the device's answer is
            # checked later and a disagreement goes to this session (post_checked)
            root, expired = spec
            st.post_expect(_d._st.OP_SESS_CLOSE, args, _d.close_expect(root, expired), (sso, _d._close_diverged,
                                                                                        sso.slot),
                           inl)
            return self._terminated(session_id, sso, de, root, expired, n)
        early = check is not None and not (v >= 0)
        if early:
            # the host knows the outcome: post the close, do the host bookkeeping that
            # needs no device answer (GC of the views with the predicted retention count,
            # the commitment record) while the hash engine finishes the chain, then await
            # the root; events go out only after the device's answer
            st.verify_deferred()
            seq = st._c.post(_d._st.OP_SESS_CLOSE, args, inl)
            self._terminate_gc(session_id, sso, de, check[1], n)
            r = await st.result_async(seq, 13, 0)
        else:
            r = await st.call_async(_d._st.OP_SESS_CLOSE, args, 13, inl, spin_busy=0)
        if guard is not None:
            # every post before the close has completed now: a prediction of this
            # session that the device refused is this terminate's error
            st.verify_deferred()
            if sso._poisoned is not None:
                raise sso._poisoned
        if r[0]:
            if r[0] == _d._st.ST_BAD_STATE:
                raise _d._lifecycle(r[1], SessionState.ACTIVE, SessionState.HANDSHAKING)
            _d._check(r, "terminate")
        root = _d._hex(r[2:10]) if r[1] else None
        if v >= 0:  # every bond of the session is released now: freeze the records, reuse the edge rows
            self.vouching.retire_session(session_id)
        # validate before publishing: a terminate whose device answer disagrees with
        # the host's view raises with nothing registered and no event emitted (the
        # commitment engine holds no record of a poisoned session)
        if early and int(r[11]) != check[1]:
            err = _d._st.StoreError(f"device GC count {int(r[11])} of session {session_id} differs from the "
                                    f"host prediction {check[1]}")
            sso._poisoned = err
            raise err
        if check is not None and audit and check[0] != root:
            # the device committed its own root; the host's view of this chain (the
            # digests it rendered and predicted) disagrees with it: the session is
            # poisoned and the terminate raises rather than hand out a root the
            # caller's records do not hash to
            err = _d._st.StoreError(f"device Merkle root {root} of session {session_id} differs from the host "
                                    f"prediction {check[0]}")
            sso._poisoned = err
            raise err
        if early:
            if root is not None:
                self.commitment.register(sso)
            self._terminate_events(session_id, root)
            return root
        return self._terminated(session_id, sso, de, root, int(r[11]), n)

    def _terminate_checked(self, session_id: str, sso, r: tuple, check: tuple) -> Optional[str]:
        """The device's answer to a terminate posted with the host's prediction
        ``check`` = (root, GC count) of a session with no liability rows: validate
        (speculations, status, GC count, root), then register and publish."""
        _d = _device_mod()
        st = self._store
        st.verify_deferred()  # every post before the close has completed now
        if sso._poisoned is not None:
            raise sso._poisoned
        if r[0]:
            if r[0] == _d._st.ST_BAD_STATE:
                raise _d._lifecycle(r[1], SessionState.ACTIVE, SessionState.HANDSHAKING)
            _d._check(r, "terminate")
        root = _d._hex(r[2:10]) if r[1] else None
        if int(r[11]) != check[1]:
            err = _d._st.StoreError(f"device GC count {int(r[11])} of session {session_id} differs from the "
                                    f"host prediction {check[1]}")
            sso._poisoned = err
            raise err
        if sso.config.enable_audit and check[0] != root:
            err = _d._st.StoreError(f"device Merkle root {root} of session {session_id} differs from the host "
                                    f"prediction {check[0]}")
            sso._poisoned = err
            raise err
        if root is not None:
            self.commitment.register(sso)
        self._terminate_events(session_id, root)
        return root

    def _terminated(self, session_id: str, sso, de, root: Optional[str], expired: int, n: int) -> Optional[str]:
        """Host bookkeeping after a device close: commitment, GC, events."""
        self._terminate_bookkeeping(session_id, sso, de, bool(root), expired, n)
        self._terminate_events(session_id, root)
        return root

    def _terminate_bookkeeping(self, session_id: str, sso, de, committed: bool, expired: int, n: int) -> None:
        """Commitment record and GC of a device close."""
        if committed:
            self.commitment.register(sso)
        self._terminate_gc(session_id, sso, de, expired, n)

    def _terminate_gc(self, session_id: str, sso, de, expired: int, n: int) -> None:
        """GC of a device close's host views (no device answer needed)."""
        # the device counts the deltas past retention (result word 12); with none
        # expired the host GC has nothing to prune and needs no walk over the views
        # a VFS nothing ever built holds no files: the collector has nothing to purge
        self.gc.collect(session_id=session_id, vfs=sso.vfs_if_built(), delta_engine=de if expired else None,
                        delta_count=de.turn_count if expired else n)

    def _terminate_events(self, session_id: str, root: Optional[str]) -> None:
        if self.event_bus is not None:
            from hypervisor.observability.event_bus import EventType

            self._emit(EventType.SESSION_TERMINATED, session_id, merkle_root=root)
            if root:
                self._emit(EventType.AUDIT_COMMITTED, session_id, merkle_root=root)
            self._emit(EventType.AUDIT_GC_COLLECTED, session_id)
            self._emit(EventType.SESSION_ARCHIVED, session_id)

    async def run_pipelines(self, specs, n: Optional[int] = None):
        """Run governance pipelines for many sessions at once on the device store
        (create → joins → activate → audit deltas → saga steps → terminate): one
        :class:`~agent_hypervisor_amd.models.store_pipeline.PipelineSpec` per
        session, or one spec and ``n``.  The sessions are ordinary sessions of this
        hypervisor afterwards (views built on first use).  Returns a
        :class:`~agent_hypervisor_amd.models.store_pipeline.PipelineRun`."""
        from agent_hypervisor_amd.models import store_pipeline

        return store_pipeline.run(self, specs, n)

    def counters(self) -> dict:
        """``/api/v1/stats`` counters: ``total_sessions``, ``active_sessions``,
        ``total_participants``, ``active_sagas``, ``total_sagas``, ``total_vouches``.
        Device-backed: reduced on the device over the hypervisor's rows (O(1) store
        commands, no snapshot or view per session); host engines: from the objects
        (reference api/server.py:144-163)."""
        if self._store is not None:
            return _device_mod().counters(self)
        ms = list(self._sessions.values())
        sagas = [g for m in ms for g in m.saga.sagas]
        return {"total_sessions": len(ms),
                "active_sessions": sum(1 for m in ms if m.sso.state.value not in ("archived", "terminating")),
                "total_participants": sum(m.sso.participant_count for m in ms),
                "active_sagas": sum(1 for g in sagas if g.state.value in ("running", "compensating")),
                "total_sagas": len(sagas), "total_vouches": len(self.vouching.records())}

    def get_session(self, session_id: str) -> Optional[ManagedSession]:
        return self._sessions.get(session_id)

    # -- behaviour verification --------------------------------------------------
    async def verify_behavior(
        self,
        session_id: str,
        agent_did: str,
        claimed_embedding: Any,
        observed_embedding: Any,
        action_id: Optional[str] = None,
    ) -> Optional[Any]:
        if not self.cmvk:
            return None
        result = self.cmvk.check_behavioral_drift(
            agent_did=agent_did,
            session_id=session_id,
            claimed_embedding=claimed_embedding,
            observed_embedding=observed_embedding,
            action_id=action_id,
        )
        if result.should_slash:
            managed = self._get_session(session_id)
            participant = managed.sso.get_participant(agent_did)
            scores = {p.agent_did: p.sigma_eff for p in managed.sso.participants}
            slash = self.slashing.slash(
                vouchee_did=agent_did,
                session_id=session_id,
                vouchee_sigma=participant.sigma_eff,
                risk_weight=0.95,
                reason=f"CMVK drift: {result.drift_score:.3f} ({result.severity.value})",
                agent_scores=scores,
            )
            if self.demote_on_slash:
                for p in managed.sso.participants:
                    if p.agent_did in scores:
                        new_ring = max(p.ring, self.ring_enforcer.compute_ring(scores[p.agent_did]), key=int)
                        if self._store is not None:
                            managed.sso.set_sigma(p.agent_did, scores[p.agent_did], new_ring)
                        else:
                            p.sigma_eff = scores[p.agent_did]
                            p.ring = new_ring
            if self.nexus:
                self.nexus.report_slash(
                    agent_did=agent_did,
                    reason=f"Behavioral drift: {result.drift_score:.3f}",
                    severity="critical" if result.drift_score >= 0.75 else "high",
                )
            if self.event_bus is not None:
                from hypervisor.observability.event_bus import EventType

                self._emit(EventType.BEHAVIOR_DRIFT, session_id, agent_did, drift=result.drift_score)
                self._emit(EventType.SLASH_EXECUTED, session_id, agent_did, slash_id=slash.slash_id)
            logger.warning("Agent %s slashed: drift=%.3f", agent_did, result.drift_score)
        return result

    # -- queries ------------------------------------------------------------------
    @property
    def sessions(self) -> list[ManagedSession]:
        """Every managed session (including archived ones), in creation order."""
        return list(self._sessions.values())

    def find_saga(self, saga_id: str):
        """(managed session, saga) owning ``saga_id``, or (None, None).  Saga ids are
        minted by the views, so batched sessions whose views were never built are
        not searched (and not built)."""
        for m in self._sessions.built_values():
            s = m.saga.get_saga(saga_id)
            if s is not None:
                return m, s
        return None, None

    def verify_audit(self, session_ids: Optional[list[str]] = None, device: Optional[str] = None,
                     checkpoints=(), source: str = "store"):
        """Batched audit of many sessions at once: every delta chain (K10), every
        committed Merkle root (K09), every VFS file against its edit log (K11) and
        the goal hashes of the given ``CheckpointManager`` s (K12) — see
        :mod:`hypervisor.audit.batch_verify`.  ``device`` defaults to the GPU for
        large batches (and to the store's device for a device-backed hypervisor).

        ``source``: ``"store"`` (default) verifies a device-backed session's audit
        where it lives — the records in the store's payload arena and the resident
        digests, nothing re-rendered or uploaded; ``"views"`` re-renders the
        Python delta views instead (which also flags edits made to those objects)."""
        from hypervisor.audit.batch_verify import verify_audit

        sessions = self.sessions if session_ids is None else [self._get_session(s) for s in session_ids]
        roots = {c.session_id: c.merkle_root for c in self.commitment.all_commitments()}
        if device is None and self._store is not None and self._store.device.type == "cuda":
            device = str(self._store.device)
        store = self._store if source == "store" else None
        return verify_audit(sessions, roots, device=device, checkpoints=checkpoints, store=store)

    @property
    def active_sessions(self) -> list[ManagedSession]:
        ms = list(self._sessions.values())
        snaps = self.snapshots(ms)
        return [m for m, sn in zip(ms, snaps) if sn.state.value not in ("archived", "terminating")]

    def snapshots(self, managed: Optional[list] = None, parts: bool = False) -> list:
        """:class:`~hypervisor.session.snapshot.SessionSnapshot` of each session (all by
        default, creation order); device-backed: O(1) store commands for any count
        (batched-pipeline sessions are read without building their views)."""
        if self._store is not None:
            from hypervisor import _device

            if managed is None:  # batches are read from their row arrays, no views built
                out = []
                for kind, seg in self._sessions.segments():
                    if kind == "own":
                        out.extend(_device.snapshots(self._store, [m.sso for m in seg], parts))
                    else:
                        out.extend(_device.snapshots_rows(self._store, *seg.rows(), parts))
                return out
            rows = [m.row if isinstance(m, LazyManagedSession) else m.sso for m in managed]
            return _device.snapshots(self._store, rows, parts)
        ms = list(self._sessions.values()) if managed is None else list(managed)
        from hypervisor.session.snapshot import SessionSnapshot

        return [SessionSnapshot.of(m.sso, parts) for m in ms]

    def saga_summaries(self, managed: Optional[list] = None) -> list[dict]:
        """Every saga of the given sessions with its step rows, as plain dicts
        (``state`` values, timestamps, retry counts); device-backed: one column
        gather per field."""
        from hypervisor._clock import from_us
        from hypervisor.saga.state_machine import SagaState, StepState

        if managed is None and self._store is not None:  # batches: from their rows, no views built
            out = []
            for kind, seg in self._sessions.segments():
                if kind == "own":
                    out.extend(self.saga_summaries(seg))
                    continue
                built = [seg.views[i] for i in sorted(seg.views)]
                out.extend(self.saga_summaries(built))
                rest = [i for i in seg.index.values() if i not in seg.views]
                gi, ti = seg.saga_row_slots(rest)
                if gi:
                    rows = self._store.gather({"g_state": gi, "g_created": gi, "g_completed": gi, "t_state": ti,
                                               "t_retry": ti, "t_started": ti, "t_completed": ti})
                    out.extend(seg.saga_summaries(rows, rest))
            return out
        ms = list(self._sessions.values()) if managed is None else list(managed)
        sagas = [g for m in ms for g in m.saga.sagas]
        out = []
        if self._store is not None and sagas:
            from hypervisor import _device

            rows = _device.saga_rows(self._store, sagas)
            gst, sst = list(SagaState), list(StepState)
            k = 0
            for i, g in enumerate(sagas):
                steps = []
                for x in g.steps:
                    t0, t1 = int(rows["t_started"][k]), int(rows["t_completed"][k])
                    steps.append({"step_id": x.step_id, "action_id": x.action_id, "agent_did": x.agent_did,
                                  "state": sst[int(rows["t_state"][k]) & 0xFF].value,
                                  "retry_count": int(rows["t_retry"][k]), "error": x.error,
                                  "started_at": from_us(t0) if t0 else None,
                                      "completed_at": from_us(t1) if t1 else None})
                    k += 1
                c1 = int(rows["g_completed"][i])
                out.append({"saga_id": g.saga_id, "session_id": g.session_id,
                            "state": gst[int(rows["g_state"][i]) & 0xFF].value, "error": g.error,
                            "created_at": from_us(int(rows["g_created"][i])),
                            "completed_at": from_us(c1) if c1 else None, "steps": steps})
            return out
        for g in sagas:
            out.append({"saga_id": g.saga_id, "session_id": g.session_id, "state": g.state.value, "error": g.error,
                        "created_at": g.created_at, "completed_at": g.completed_at,
                        "steps": [{"step_id": x.step_id, "action_id": x.action_id, "agent_did": x.agent_did,
                                   "state": x.state.value, "retry_count": x.retry_count, "error": x.error,
                                   "started_at": x.started_at, "completed_at": x.completed_at} for x in g.steps]})
        return out

    def _get_session(self, session_id: str) -> ManagedSession:
        m = self._sessions.get(session_id)
        if m is None:
            raise ValueError(f"Session {session_id} not found")
        return m

    # -- MI355X batched pipeline ------------------------------------------------------
    def pipeline_batch(self, n_sessions: int, **kwargs):
        """Run the reference pipeline for ``n_sessions`` new sessions in one device
        launch, written into this hypervisor's store (one device state: they are
        ordinary sessions afterwards — ``get_session``, terminate, ``verify_audit``,
        checkpoints).  See :func:`agent_hypervisor_amd.models.store_template.run`
        (``agents``, ``session_agent``, ``deltas``, ``changes``, ``now_us``,
        ``config``); returns a :class:`~agent_hypervisor_amd.models.store_pipeline.PipelineRun`."""
        from agent_hypervisor_amd.models import store_template

        run = store_template.run(self, n_sessions, **kwargs)
        self.batched_sessions += n_sessions
        return run
