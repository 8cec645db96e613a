"""The hypervisor's session table: session id → ManagedSession, in creation order.

Sessions a batched store pipeline wrote (:meth:`hypervisor.Hypervisor.run_pipelines`)
are held per batch — the batch keeps an id → index map — and get Python views
only on first use.  Until then the batch owns their store rows, and it returns
the rows of never-used sessions when it goes; registering 10⁵ batched sessions
costs two dict inserts each and creates no per-session object.

Mapping surface used by the hypervisor and its tools: ``get``, ``[]``, ``in``,
``len``, iteration (ids), ``values``, ``items``, ``pop`` and ``[sid] = m`` (an
ordinary session).  ``values()`` yields the built view of a batched session, or
a transient :class:`hypervisor.core.LazyManagedSession` proxy for one that has
none yet (its attributes build the views).
"""

from __future__ import annotations

from array import array
from typing import Iterator, Optional

import numpy as np


class SessionTable:
    __slots__ = ("_own", "_segs", "_lazy", "_slots", "_pos", "saga_rows", "_bcache")

    def __init__(self) -> None:
        self._own: dict = {}   # ordinary (and restored) sessions
        self._segs: list = []  # creation order: a list of own ids, or a batch
        self._lazy: dict = {}  # batched session id → its batch
        # device rows of the own sessions in insertion order (-1: host session or
        # removed) and of the sagas created through their orchestrators: the
        # counters views reduce these on the device without walking the sessions
        self._slots = array("q")
        self._pos: dict = {}
        self.saga_rows = array("q")
        self._bcache: dict = {}  # id(batch) → (live count, its live session rows)

    def __len__(self) -> int:
        return len(self._own) + len(self._lazy)

    def __contains__(self, sid) -> bool:
        return sid in self._own or sid in self._lazy

    def get(self, sid, default=None):
        m = self._own.get(sid)
        if m is not None:
            return m
        b = self._lazy.get(sid)
        if b is None:
            return default
        m = b.view(b.index[sid])
        orch = m.saga
        if getattr(orch, "_reg", False) is None:  # sagas created on it later are counted too
            orch._reg = self.saga_rows
        return m

    def __getitem__(self, sid):
        m = self.get(sid)
        if m is None:
            raise KeyError(sid)
        return m

    def __setitem__(self, sid, m) -> None:
        if sid in self._lazy:
            raise ValueError(f"session {sid} belongs to a batch")
        if sid not in self._own:
            if not self._segs or not isinstance(self._segs[-1], list):
                self._segs.append([])
            self._segs[-1].append(sid)
            self._pos[sid] = len(self._slots)
            self._slots.append(getattr(m.sso, "slot", -1))
        self._own[sid] = m

    def add_batch(self, batch, ids: list) -> None:
        """Register the sessions ``ids`` of ``batch`` (``batch.index`` maps them)."""
        self._segs.append(batch)
        self._lazy.update(dict.fromkeys(ids, batch))

    def pop(self, sid, default=None):
        m = self._own.pop(sid, None)
        if m is not None:
            k = self._pos.pop(sid, None)
            if k is not None:
                self._slots[k] = -1
            for seg in self._segs:
                if isinstance(seg, list) and sid in seg:
                    seg.remove(sid)
                    break
            return m
        b = self._lazy.pop(sid, None)
        if b is None:
            return default
        return b.forget(b.index.pop(sid))

    def __iter__(self) -> Iterator[str]:
        own = self._own
        for seg in self._segs:
            if isinstance(seg, list):
                yield from (sid for sid in seg if sid in own)
            else:
                yield from seg.index

    keys = __iter__

    def values(self):
        own = self._own
        for seg in self._segs:
            if isinstance(seg, list):
                for sid in seg:
                    m = own.get(sid)
                    if m is not None:
                        yield m
            else:
                yield from seg.entries()

    def built_values(self):
        """The sessions that have Python views (ordinary ones and batched ones
        already used) — what a search for an id the views minted needs."""
        own = self._own
        for seg in self._segs:
            if isinstance(seg, list):
                for sid in seg:
                    m = own.get(sid)
                    if m is not None:
                        yield m
            else:
                yield from (seg.views[i] for i in sorted(seg.views))

    def items(self):
        for sid, m in zip(self, self.values()):
            yield sid, m

    def segments(self):
        """(kind, payload) runs in creation order: ("own", [ManagedSession]) or
        ("batch", batch) — lets batched views read a batch's rows without views."""
        own = self._own
        for seg in self._segs:
            if isinstance(seg, list):
                ms = [own[sid] for sid in seg if sid in own]
                if ms:
                    yield "own", ms
            elif seg.index:
                yield "batch", seg

    def batches(self) -> list:
        """Every batch segment, including batches whose sessions have all left the
        table (their unbuilt rows may still wait in ``dead`` for release)."""
        return [seg for seg in self._segs if not isinstance(seg, list)]

    def prune_batches(self) -> None:
        """Drop batch segments with no session left in the table and no built view
        (call after their ``dead`` rows were released)."""
        keep = [seg for seg in self._segs if isinstance(seg, list) or seg.index or seg.views]
        for seg in self._segs:
            if not isinstance(seg, list) and not (seg.index or seg.views):
                self._bcache.pop(id(seg), None)
        self._segs = keep

    def batch_of(self, sid) -> Optional[object]:
        return self._lazy.get(sid)

    # -- device rows (counter views) ---------------------------------------------
    def _batch_rows(self, seg) -> tuple:
        """(live session rows, live saga rows) of a batch, cached until it loses a session."""
        n = len(seg.index)
        c = self._bcache.get(id(seg))
        if c is None or c[0] != n or c[3] is not seg:
            idx = np.fromiter(seg.index.values(), dtype=np.int64, count=n)
            gs = np.asarray(seg.gslots, dtype=np.int64)
            goff = getattr(seg, "goff", None)
            if goff is not None:  # restored batch: any number of sagas per session
                g0, g1 = goff[idx], goff[idx + 1]
                cnt = (g1 - g0).astype(np.int64)
                k = int(cnt.sum())
                rows = gs[np.repeat(g0 - np.concatenate([[0], np.cumsum(cnt)[:-1]]), cnt) + np.arange(k)] \
                    if k else np.zeros(0, np.int64)
            else:  # pipeline batch: at most one saga per session
                rows = gs[idx]
                rows = rows[rows >= 0]
            c = (n, seg.slots[idx].astype(np.int64), rows.astype(np.int64), seg)
            self._bcache[id(seg)] = c
        return c[1], c[2]

    def session_slots(self) -> np.ndarray:
        """Device session rows of every session in the table (int64; host sessions
        have none): the own sessions' array as kept, plus each batch's live rows.
        No view is built."""
        own = np.frombuffer(self._slots, dtype=np.int64) if len(self._slots) else np.zeros(0, np.int64)
        parts = [own[own >= 0]]
        for seg in self._segs:
            if not isinstance(seg, list) and seg.index:
                parts.append(self._batch_rows(seg)[0])
        return np.concatenate(parts) if len(parts) > 1 else parts[0]

    def batch_saga_rows(self) -> np.ndarray:
        """Saga rows the batches wrote for their sessions still in the table, int64."""
        out = [self._batch_rows(seg)[1] for seg in self._segs if not isinstance(seg, list) and seg.index]
        return np.concatenate(out) if out else np.zeros(0, np.int64)

    def forget_sagas(self, rows) -> None:
        """Drop saga rows of sessions that left the table (bulk: one pass)."""
        drop = set(int(r) for r in rows)
        if drop:
            self.saga_rows = array("q", (r for r in self.saga_rows if r not in drop))
