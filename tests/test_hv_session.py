"""Shared sessions: lifecycle, participants, VFS substrate, snapshots, vector
clocks, intent locks and isolation levels (reference session/*.py; behaviours
listed in SURVEY §2 C01–C08)."""

from __future__ import annotations

import hashlib

import pytest

from hypervisor.models import ConsistencyMode, ExecutionRing, SessionConfig, SessionState
from hypervisor.session import SessionLifecycleError, SessionParticipantError, SharedSessionObject
from hypervisor.session.intent_locks import DeadlockError, IntentLockManager, LockContentionError, LockIntent
from hypervisor.session.isolation import IsolationLevel
from hypervisor.session.sso import SessionVFS, VFSPermissionError
from hypervisor.session.vector_clock import CausalViolationError, VectorClock, VectorClockManager


def _sso(**cfg) -> SharedSessionObject:
    return SharedSessionObject(SessionConfig(**cfg), creator_did="did:creator")


# ---------------------------------------------------------------- lifecycle


class TestLifecycle:
    def test_initial_state_and_ids(self):
        s = _sso()
        assert s.state == SessionState.CREATED
        assert s.session_id.startswith("session:")
        assert s.vfs_namespace == f"/sessions/{s.session_id}"
        assert s.terminated_at is None and s.participant_count == 0

    def test_full_state_walk(self):
        s = _sso()
        s.begin_handshake()
        s.join("did:a")
        s.activate()
        assert s.state == SessionState.ACTIVE
        s.terminate()
        assert s.state == SessionState.TERMINATING and s.terminated_at is not None
        s.archive()
        assert s.state == SessionState.ARCHIVED

    def test_terminate_from_handshaking_allowed(self):
        s = _sso()
        s.begin_handshake()
        s.terminate()
        assert s.state == SessionState.TERMINATING

    @pytest.mark.parametrize("op", ["activate", "terminate", "archive"])
    def test_invalid_from_created(self, op):
        with pytest.raises(SessionLifecycleError, match="not allowed in state created"):
            getattr(_sso(), op)()

    def test_double_handshake_rejected(self):
        s = _sso()
        s.begin_handshake()
        with pytest.raises(SessionLifecycleError):
            s.begin_handshake()

    def test_activate_needs_participants(self):
        s = _sso()
        s.begin_handshake()
        with pytest.raises(SessionLifecycleError, match="no participants"):
            s.activate()

    def test_join_requires_handshaking_or_active(self):
        s = _sso()
        with pytest.raises(SessionLifecycleError):
            s.join("did:a")
        s.begin_handshake()
        s.join("did:a")
        s.activate()
        s.join("did:b")  # late join while active
        s.terminate()
        with pytest.raises(SessionLifecycleError):
            s.join("did:c")

    def test_repr(self):
        assert "state=created" in repr(_sso())


class TestParticipants:
    def test_duplicate_join(self):
        s = _sso()
        s.begin_handshake()
        s.join("did:a")
        with pytest.raises(SessionParticipantError, match="already in session"):
            s.join("did:a")

    def test_capacity(self):
        s = _sso(max_participants=2)
        s.begin_handshake()
        s.join("did:a")
        s.join("did:b")
        with pytest.raises(SessionParticipantError, match="capacity"):
            s.join("did:c")

    def test_min_sigma_applies_outside_sandbox_only(self):
        s = _sso(min_sigma_eff=0.6)
        s.begin_handshake()
        s.join("did:sandboxed", sigma_eff=0.1)  # ring 3 is always admissible
        with pytest.raises(SessionParticipantError, match="below minimum"):
            s.join("did:low", sigma_eff=0.5, ring=ExecutionRing.RING_2_STANDARD)
        p = s.join("did:ok", sigma_eff=0.7, ring=ExecutionRing.RING_2_STANDARD)
        assert p.ring == ExecutionRing.RING_2_STANDARD

    def test_leave_deactivates_and_frees_capacity(self):
        s = _sso(max_participants=1)
        s.begin_handshake()
        s.join("did:a")
        s.leave("did:a")
        assert s.participant_count == 0 and s.participants == []
        s.join("did:b")
        with pytest.raises(SessionParticipantError):
            s.join("did:a")  # a left participant cannot rejoin under the same DID

    def test_get_and_update_ring(self):
        s = _sso()
        s.begin_handshake()
        s.join("did:a")
        s.update_ring("did:a", ExecutionRing.RING_1_PRIVILEGED)
        assert s.get_participant("did:a").ring == ExecutionRing.RING_1_PRIVILEGED
        with pytest.raises(SessionParticipantError, match="not in session"):
            s.get_participant("did:zz")

    def test_force_consistency_mode(self):
        s = _sso()
        s.force_consistency_mode(ConsistencyMode.STRONG)
        assert s.consistency_mode == ConsistencyMode.STRONG


# ---------------------------------------------------------------------- VFS


class TestVFS:
    def test_write_read_create_update(self):
        v = SessionVFS("s1")
        e1 = v.write("/a.txt", "one", "did:a")
        assert e1.operation == "create" and e1.path == "/sessions/s1/a.txt"
        assert e1.content_hash == hashlib.sha256(b"one").hexdigest() and e1.previous_hash is None
        e2 = v.write("a.txt", "two", "did:b")
        assert e2.operation == "update" and e2.previous_hash == e1.content_hash
        assert v.read("/a.txt") == "two"
        assert v.read("/missing") is None

    def test_namespaced_paths_pass_through(self):
        v = SessionVFS("s1")
        v.write("/sessions/s1/x", "1", "d")
        assert v.read("/x") == "1"
        assert v.list_files() == ["/x"]

    def test_custom_namespace(self):
        v = SessionVFS("s1", namespace="/ns")
        v.write("f", "x", "d")
        assert v.list_files() == ["/f"]

    def test_delete(self):
        v = SessionVFS("s1")
        v.write("/a", "x", "d")
        e = v.delete("/a", "d")
        assert e.operation == "delete" and e.previous_hash == hashlib.sha256(b"x").hexdigest()
        assert v.file_count == 0
        with pytest.raises(FileNotFoundError):
            v.delete("/a", "d")

    def test_permissions(self):
        v = SessionVFS("s1")
        v.write("/secret", "s", "did:owner")
        v.set_permissions("/secret", {"did:owner"}, "did:owner")
        assert v.get_permissions("/secret") == {"did:owner"}
        assert v.read("/secret", "did:owner") == "s"
        assert v.read("/secret") == "s"  # anonymous read skips the ACL
        with pytest.raises(VFSPermissionError):
            v.read("/secret", "did:other")
        with pytest.raises(VFSPermissionError):
            v.write("/secret", "x", "did:other")
        with pytest.raises(VFSPermissionError):
            v.delete("/secret", "did:other")
        v.clear_permissions("/secret")
        v.write("/secret", "x", "did:other")

    def test_delete_drops_acl(self):
        v = SessionVFS("s1")
        v.write("/f", "x", "a")
        v.set_permissions("/f", {"a"}, "a")
        v.delete("/f", "a")
        assert v.get_permissions("/f") is None
        v.write("/f", "y", "b")

    def test_edit_log_and_attribution(self):
        v = SessionVFS("s1")
        v.write("/a", "1", "x")
        v.write("/b", "2", "y")
        v.write("/a", "3", "x")
        assert [e.operation for e in v.edit_log] == ["create", "create", "update"]
        assert len(v.edits_by_agent("x")) == 2
        log = v.edit_log
        log.clear()
        assert len(v.edit_log) == 3  # copy returned

    def test_snapshots(self):
        v = SessionVFS("s1")
        v.write("/a", "1", "x")
        v.set_permissions("/a", {"x"}, "x")
        sid = v.create_snapshot()
        v.write("/a", "2", "x")
        v.write("/b", "3", "x")
        v.clear_permissions("/a")
        v.restore_snapshot(sid, "x")
        assert v.read("/a") == "1" and v.read("/b") is None and v.get_permissions("/a") == {"x"}
        assert v.edit_log[-1].operation == "restore"
        assert v.list_snapshots() == [sid] and v.snapshot_count == 1
        v.delete_snapshot(sid)
        with pytest.raises(KeyError):
            v.restore_snapshot(sid, "x")
        with pytest.raises(KeyError):
            v.delete_snapshot(sid)

    def test_named_snapshot_isolated_from_later_writes(self):
        v = SessionVFS("s1")
        v.write("/a", "1", "x")
        v.create_snapshot("snap-1")
        v.write("/a", "2", "x")
        v.restore_snapshot("snap-1", "x")
        v.write("/a", "3", "x")
        v.restore_snapshot("snap-1", "x")
        assert v.read("/a") == "1"

    def test_total_bytes_and_purge(self):
        v = SessionVFS("s1")
        v.write("/a", "héllo", "x")
        v.create_snapshot()
        assert v.total_bytes == len("héllo".encode())
        assert v.purge() == 1
        assert v.file_count == 0 and v.snapshot_count == 0


class TestSessionSnapshots:
    def test_requires_active(self):
        s = _sso()
        s.begin_handshake()
        with pytest.raises(SessionLifecycleError):
            s.create_vfs_snapshot()

    def test_snapshot_roundtrip_records_participants(self):
        s = _sso()
        s.begin_handshake()
        s.join("did:a", sigma_eff=0.7)
        s.activate()
        s.vfs.write("/f", "1", "did:a")
        snap = s.create_vfs_snapshot()
        s.vfs.write("/f", "2", "did:a")
        s.restore_vfs_snapshot(snap, "did:a")
        assert s.vfs.read("/f") == "1"
        assert s._vfs_snapshots[snap]["participant_states"]["did:a"]["sigma_eff"] == 0.7


# ------------------------------------------------------------ vector clocks


class TestVectorClock:
    def test_tick_get_merge(self):
        a, b = VectorClock(), VectorClock()
        a.tick("x")
        a.tick("x")
        b.tick("y")
        m = a.merge(b)
        assert m.get("x") == 2 and m.get("y") == 1 and m.get("z") == 0
        assert a.get("y") == 0  # merge is pure

    def test_ordering(self):
        a, b = VectorClock(), VectorClock()
        a.tick("x")
        b = a.copy()
        b.tick("y")
        assert a.happens_before(b) and not b.happens_before(a)
        assert not a.happens_before(a)
        c = VectorClock()
        c.tick("z")
        assert a.is_concurrent(c) and c.is_concurrent(a)

    def test_equality_ignores_zero_entries(self):
        a, b = VectorClock(), VectorClock()
        a.tick("x")
        b.tick("x")
        assert a == b
        b.tick("y")
        assert a != b


class TestVectorClockManager:
    def test_write_then_read(self):
        m = VectorClockManager()
        c = m.write("/f", "a")
        assert c.get("a") == 1 and m.tracked_paths == 1
        r = m.read("/f", "b")
        assert r.get("a") == 1 and m.get_agent_clock("b").get("a") == 1

    def test_stale_write_rejected_in_strict_mode(self):
        m = VectorClockManager()
        m.write("/f", "a")
        m.read("/f", "b")
        m.write("/f", "a")  # path moves ahead of b's view
        with pytest.raises(CausalViolationError, match="stale state"):
            m.write("/f", "b")
        assert m.conflict_count == 1
        m.write("/f", "b", strict=False)
        m.read("/f", "b")
        m.write("/f", "b")

    def test_first_write_by_anyone_allowed(self):
        m = VectorClockManager()
        m.write("/f", "x")
        m.write("/g", "y")  # fresh path, empty path clock

    def test_unknown_clock_queries_empty(self):
        m = VectorClockManager()
        assert m.get_path_clock("/none").clocks == {}
        assert m.get_agent_clock("nobody").clocks == {}


# -------------------------------------------------------------- intent locks


class TestIntentLocks:
    def test_read_read_shared(self):
        m = IntentLockManager()
        m.acquire("a", "s", "/r", LockIntent.READ)
        m.acquire("b", "s", "/r", LockIntent.READ)
        assert m.active_lock_count == 2

    @pytest.mark.parametrize("held,want", [("read", "write"), ("write", "read"), ("write", "write"),
                                           ("exclusive", "read"), ("read", "exclusive")])
    def test_conflicts(self, held, want):
        m = IntentLockManager()
        m.acquire("a", "s", "/r", LockIntent(held))
        with pytest.raises(LockContentionError, match="Lock contention"):
            m.acquire("b", "s", "/r", LockIntent(want))

    def test_same_agent_never_conflicts(self):
        m = IntentLockManager()
        m.acquire("a", "s", "/r", LockIntent.EXCLUSIVE)
        m.acquire("a", "s", "/r", LockIntent.WRITE)

    def test_release_paths(self):
        m = IntentLockManager()
        l1 = m.acquire("a", "s", "/r", LockIntent.WRITE)
        m.acquire("a", "s", "/q", LockIntent.WRITE)
        m.acquire("b", "s2", "/z", LockIntent.READ)
        m.release(l1.lock_id)
        m.release("unknown")  # no-op
        assert not l1.is_active
        m.acquire("c", "s", "/r", LockIntent.WRITE)
        assert m.release_agent_locks("a", "s") == 1
        assert m.release_session_locks("s") == 1
        assert m.active_lock_count == 1

    def test_queries(self):
        m = IntentLockManager()
        m.acquire("a", "s", "/r", LockIntent.READ)
        m.acquire("b", "s", "/r", LockIntent.READ)
        assert len(m.get_resource_locks("/r")) == 2
        assert len(m.get_agent_locks("a", "s")) == 1
        assert m.contention_points == [] or isinstance(m.contention_points, list)

    def test_deadlock_detection_with_wait_graph(self):
        m = IntentLockManager(record_waits=True)
        m.acquire("a", "s", "/x", LockIntent.WRITE)
        m.acquire("b", "s", "/y", LockIntent.WRITE)
        with pytest.raises(LockContentionError):
            m.acquire("a", "s", "/y", LockIntent.WRITE)  # a waits on b
        with pytest.raises(DeadlockError, match="Deadlock"):
            m.acquire("b", "s", "/x", LockIntent.WRITE)  # b would wait on a


class TestIsolation:
    def test_traits(self):
        assert IsolationLevel.SNAPSHOT.allows_concurrent_writes
        assert not IsolationLevel.SNAPSHOT.requires_vector_clocks
        assert IsolationLevel.SERIALIZABLE.requires_vector_clocks
        assert IsolationLevel.SERIALIZABLE.requires_intent_locks
        assert not IsolationLevel.SERIALIZABLE.allows_concurrent_writes
        assert IsolationLevel.READ_COMMITTED.requires_vector_clocks
        assert not IsolationLevel.READ_COMMITTED.requires_intent_locks
        assert [l.coordination_cost for l in IsolationLevel] == ["low", "moderate", "high"]
