"""Session-scoped virtual file system (the SSO "state substrate").

Parity target: reference ``session/sso.py:29-216``.  Observable rules:

* paths resolve into ``/sessions/<id>``; a path already under the namespace is
  kept verbatim, anything else has leading ``/`` stripped and is prefixed;
* a path with a permission entry is restricted to that agent set; ``write``,
  ``delete`` and ``read`` *with* an ``agent_did`` are checked;
* every mutation appends a :class:`VFSEdit` carrying SHA-256 content hashes
  (computed by the native core, ``agent_hypervisor_amd._C.sha256_hex``);
* snapshots deep-copy files **and** permissions (copy-on-write semantics).

Additions beyond the reference: :meth:`SessionVFS.purge` (used by the GC, which
in the reference silently failed to delete anything — SURVEY Appendix A Q01) and
``total_bytes`` for GC accounting.
"""

from __future__ import annotations

import copy
from dataclasses import dataclass, field
from datetime import datetime
from typing import Optional

from agent_hypervisor_amd._native import C as _C
from hypervisor._clock import now as _now

_sha256_hex = _C.sha256_hex


def _hash(content: str) -> str:
    return _sha256_hex(content)


@dataclass
class VFSEdit:
    path: str
    operation: str  # create | update | delete | permission | restore
    agent_did: str
    timestamp: datetime = field(default_factory=_now)
    content_hash: Optional[str] = None
    previous_hash: Optional[str] = None


class VFSPermissionError(Exception):
    """An agent touched a path whose permission set excludes it."""


class SessionVFS:
    """In-memory, namespaced file store with attribution, ACLs and snapshots."""

    def __init__(self, session_id: str, namespace: Optional[str] = None):
        self.session_id = session_id
        self.namespace = namespace or f"/sessions/{session_id}"
        self._files: dict[str, str] = {}
        self._permissions: dict[str, set[str]] = {}
        self._edit_log: list[VFSEdit] = []
        self._snapshots: dict[str, dict[str, dict]] = {}

    # -- path handling -------------------------------------------------
    def _resolve(self, path: str) -> str:
        ns = self.namespace
        if path.startswith(ns):
            return path
        return ns + "/" + path.lstrip("/")

    def _check_permission(self, full_path: str, agent_did: str) -> None:
        acl = self._permissions.get(full_path)
        if acl is not None and agent_did not in acl:
            raise VFSPermissionError(f"Agent {agent_did} not permitted to access {full_path}")

    def _log(self, edit: VFSEdit) -> VFSEdit:
        self._edit_log.append(edit)
        return edit

    # -- file operations ----------------------------------------------
    def write(self, path: str, content: str, agent_did: str) -> VFSEdit:
        full = self._resolve(path)
        self._check_permission(full, agent_did)
        old = self._files.get(full)
        self._files[full] = content
        if old is None:
            return self._log(VFSEdit(full, "create", agent_did, content_hash=_hash(content)))
        return self._log(
            VFSEdit(full, "update", agent_did, content_hash=_hash(content), previous_hash=_hash(old))
        )

    def read(self, path: str, agent_did: Optional[str] = None) -> Optional[str]:
        full = self._resolve(path)
        if agent_did is not None:
            self._check_permission(full, agent_did)
        return self._files.get(full)

    def delete(self, path: str, agent_did: str) -> VFSEdit:
        full = self._resolve(path)
        if full not in self._files:
            raise FileNotFoundError(f"{full} not found in session VFS")
        self._check_permission(full, agent_did)
        old = self._files.pop(full)
        self._permissions.pop(full, None)
        return self._log(VFSEdit(full, "delete", agent_did, previous_hash=_hash(old)))

    def list_files(self) -> list[str]:
        ns = self.namespace
        n = len(ns)
        return [p[n:] for p in self._files if p.startswith(ns)]

    # -- permissions ----------------------------------------------------
    def set_permissions(self, path: str, allowed_agents: set[str], agent_did: str) -> VFSEdit:
        full = self._resolve(path)
        self._permissions[full] = set(allowed_agents)
        return self._log(VFSEdit(full, "permission", agent_did))

    def clear_permissions(self, path: str) -> None:
        self._permissions.pop(self._resolve(path), None)

    def get_permissions(self, path: str) -> Optional[set[str]]:
        return self._permissions.get(self._resolve(path))

    # -- snapshots --------------------------------------------------------
    def create_snapshot(self, snapshot_id: Optional[str] = None) -> str:
        sid = snapshot_id or _C.uuid4("snap:")
        self._snapshots[sid] = {
            "files": dict(self._files),  # str values are immutable: a shallow copy is a deep copy
            "permissions": copy.deepcopy(self._permissions),
        }
        return sid

    def restore_snapshot(self, snapshot_id: str, agent_did: str) -> None:
        snap = self._snapshots.get(snapshot_id)
        if snap is None:
            raise KeyError(f"Snapshot {snapshot_id} not found")
        self._files = dict(snap["files"])
        self._permissions = copy.deepcopy(snap["permissions"])
        self._log(VFSEdit(self.namespace, "restore", agent_did))

    def list_snapshots(self) -> list[str]:
        return list(self._snapshots)

    def delete_snapshot(self, snapshot_id: str) -> None:
        if snapshot_id not in self._snapshots:
            raise KeyError(f"Snapshot {snapshot_id} not found")
        del self._snapshots[snapshot_id]

    # -- queries ----------------------------------------------------------
    @property
    def edit_log(self) -> list[VFSEdit]:
        return list(self._edit_log)

    def edits_by_agent(self, agent_did: str) -> list[VFSEdit]:
        return [e for e in self._edit_log if e.agent_did == agent_did]

    @property
    def file_count(self) -> int:
        return len(self._files)

    @property
    def snapshot_count(self) -> int:
        return len(self._snapshots)

    @property
    def total_bytes(self) -> int:
        """UTF-8 bytes held by live files (GC accounting)."""
        return sum(len(v.encode()) for v in self._files.values())

    # -- GC hook ------------------------------------------------------------
    def purge(self) -> int:
        """Drop every live file, its ACL and all snapshots; returns files purged."""
        n = len(self._files)
        self._files = {}
        self._permissions = {}
        self._snapshots = {}
        return n
