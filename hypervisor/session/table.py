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

from typing import Iterator, Optional


class SessionTable:
    __slots__ = ("_own", "_segs", "_lazy")

    def __init__(self) -> None:
        self._own: dict = {}   # ordinary (and restored) sessions
        self._segs: list = []  # creation order: a list of own ids, or a batch
        self._lazy: dict = {}  # batched session id → its batch

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
        return b.view(b.index[sid])

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
        self._own[sid] = m

    def add_batch(self, batch, ids: list) -> None:
        """Register the sessions ``ids`` of ``batch`` (``batch.index`` maps them)."""
        self._segs.append(batch)
        self._lazy.update(dict.fromkeys(ids, batch))

    def pop(self, sid, default=None):
        m = self._own.pop(sid, None)
        if m is not None:
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

    def batch_of(self, sid) -> Optional[object]:
        return self._lazy.get(sid)
