"""Ephemeral garbage collection of terminated sessions.

Parity target: reference ``audit/gc.py:15-141`` (result/accounting formulas are
identical: ``retained_deltas = delta_count − expired``, storage after = the delta
bytes when deltas exist, else 0).

Fix: the reference called ``vfs.delete(f)`` without the
required ``agent_did``, swallowed the ``TypeError`` and reported files as purged
while keeping them.  Here the VFS is actually purged (:meth:`SessionVFS.purge`)
and the count is what was dropped; parity mode reproduces the reporting-only
behaviour.  Deltas older than the retention window are pruned through
``DeltaEngine.prune_expired`` (the hook the reference probed for but never had).
"""

from __future__ import annotations

from dataclasses import dataclass, field
from datetime import datetime, timedelta
from typing import Any, Optional

from hypervisor import config as _cfg
from hypervisor._clock import now as _now


@dataclass
class GCResult:
    session_id: str
    retained_deltas: int
    retained_hash: bool
    purged_vfs_files: int
    purged_caches: int
    storage_before_bytes: int
    storage_after_bytes: int
    gc_at: datetime = field(default_factory=_now)

    @property
    def storage_saved_bytes(self) -> int:
        return self.storage_before_bytes - self.storage_after_bytes

    @property
    def savings_pct(self) -> float:
        if self.storage_before_bytes == 0:
            return 0.0
        return self.storage_saved_bytes / self.storage_before_bytes * 100


@dataclass
class RetentionPolicy:
    delta_retention_days: int = 90
    hash_retention: str = "permanent"
    liability_snapshot: bool = True


class EphemeralGC:
    def __init__(self, policy: Optional[RetentionPolicy] = None) -> None:
        self.policy = policy or RetentionPolicy()
        self._gc_history: list[GCResult] = []
        self._purged_sessions: set[str] = set()

    def _purge_vfs(self, vfs: Any, fallback: int) -> int:
        try:
            files = vfs.list_files() if hasattr(vfs, "list_files") else []
        except Exception:
            return fallback
        if _cfg.parity_mode() or not hasattr(vfs, "purge"):
            return len(files)
        return vfs.purge()

    def collect(
        self,
        session_id: str,
        vfs: Any = None,
        delta_engine: Any = None,
        vfs_file_count: int = 0,
        cache_count: int = 0,
        delta_count: int = 0,
        estimated_vfs_bytes: int = 0,
        estimated_cache_bytes: int = 0,
        estimated_delta_bytes: int = 0,
    ) -> GCResult:
        purged = self._purge_vfs(vfs, vfs_file_count) if vfs is not None else vfs_file_count
        retained = delta_count
        if delta_engine is not None and hasattr(delta_engine, "deltas"):
            cutoff = _now() - timedelta(days=self.policy.delta_retention_days)
            expired = sum(1 for d in delta_engine.deltas if d.timestamp < cutoff)
            retained = delta_count - expired
            if expired and hasattr(delta_engine, "prune_expired") and not _cfg.parity_mode():
                delta_engine.prune_expired(self.policy.delta_retention_days)
        res = GCResult(
            session_id=session_id,
            retained_deltas=max(retained, 0),
            retained_hash=True,
            purged_vfs_files=purged,
            purged_caches=cache_count,
            storage_before_bytes=estimated_vfs_bytes + estimated_cache_bytes + estimated_delta_bytes,
            storage_after_bytes=estimated_delta_bytes if delta_count > 0 else 0,
        )
        self._gc_history.append(res)
        self._purged_sessions.add(session_id)
        return res

    def is_purged(self, session_id: str) -> bool:
        return session_id in self._purged_sessions

    def should_expire_deltas(self, delta_timestamp: datetime) -> bool:
        return delta_timestamp < _now() - timedelta(days=self.policy.delta_retention_days)

    @property
    def history(self) -> list[GCResult]:
        return list(self._gc_history)

    @property
    def purged_session_count(self) -> int:
        return len(self._purged_sessions)
