"""GovernanceStore: the device-authoritative state behind ``Hypervisor(device=...)``.

Every row of governance state the public API owns — sessions and their
participants, the audit chain (digests + canonical-JSON records), vouch bonds,
sagas and steps — lives in SoA PyTorch tensors on the HIP device (SURVEY N04;
column list: ``STORE_COLUMNS`` of ``csrc/include/ahv/store.h``).  API calls are
commands executed by a resident gfx950 worker wave (``csrc/hip/store_worker.hip``)
over a PCIe doorbell ring; the host keeps only what is not state: string
interning (DIDs / liability-session keys → dense ids), row allocators, and
Python objects the user handed in (executors, results, VFS file contents).

``device="cpu"`` runs the identical command processor (``store_exec``) inline on
CPU tensors — the host twin the CPU suite and the reference oracle run against.

One store per (process, device) is shared by every ``Hypervisor`` on it
(:func:`shared_store`): the reference benchmark builds a fresh ``Hypervisor()``
per pipeline, which must not allocate tables each time.  Rows are recycled
only once no API object refers to them (never while live); full tables grow by
doubling up to ``AHV_STORE_MAX_*`` (defaults sized for 288 GB of HBM3E).
"""

from __future__ import annotations

import atexit
import os
import struct
import threading
from typing import Optional

import numpy as np
import torch

from agent_hypervisor_amd._native import C
from agent_hypervisor_amd.utils.interner import Interner

OPS = dict(C.STORE_OPS)
globals().update(OPS)  # OP_* constants

_DTYPES = {
    "uint8_t": torch.uint8,
    "int32_t": torch.int32,
    "uint32_t": torch.int32,  # bit patterns (digest / uuid words)
    "int64_t": torch.int64,
    "double": torch.float64,
}

_NP_OF = {torch.uint8: np.dtype(np.uint8), torch.int32: np.dtype(np.int32), torch.int64: np.dtype(np.int64),
          torch.float64: np.dtype(np.float64)}

ST_OK, ST_BAD_STATE, ST_NOT_FOUND, ST_BAD_ARG, ST_SCRATCH = 0, 1, 2, 90, 91

_u64 = struct.Struct("<Q")
_d = struct.Struct("<d")
_i64_of_d = struct.Struct("<q").unpack


def dbits(x: float) -> int:
    """fp64 bit pattern as a signed int64 (store argument encoding)."""
    return _i64_of_d(_d.pack(x))[0]


def bitsd(v: int) -> float:
    return _d.unpack(_u64.pack(v & 0xFFFFFFFFFFFFFFFF))[0]


def _env_int(name: str, default: int) -> int:
    v = os.environ.get(name)
    return int(v) if v else default


def default_caps() -> dict:
    return {
        "S": _env_int("AHV_STORE_SESSIONS", 1 << 16),
        "P": _env_int("AHV_STORE_PARTICIPANTS", 32),
        "D": _env_int("AHV_STORE_DELTAS", 1 << 18),
        "E": _env_int("AHV_STORE_VOUCHES", 1 << 18),
        "V": _env_int("AHV_STORE_LIABILITY_SESSIONS", 1 << 16),
        "G": _env_int("AHV_STORE_SAGAS", 1 << 16),
        "T": _env_int("AHV_STORE_STEPS", 1 << 17),
        "X": _env_int("AHV_STORE_SCRATCH", 1 << 22),
        "B": _env_int("AHV_STORE_PAYLOAD", 1 << 26),
    }


def default_max_caps() -> dict:
    """Growth ceilings (``AHV_STORE_MAX_*``): sized for one 288 GB MI355X — a session
    row with 32 participant rows is ≈1.4 KB, a delta row 72 B + its ≈300 B record."""
    return {
        "S": _env_int("AHV_STORE_MAX_SESSIONS", 1 << 25),
        "D": _env_int("AHV_STORE_MAX_DELTAS", 1 << 28),
        "E": _env_int("AHV_STORE_MAX_VOUCHES", 1 << 28),
        "V": _env_int("AHV_STORE_MAX_LIABILITY_SESSIONS", 1 << 25),
        "G": _env_int("AHV_STORE_MAX_SAGAS", 1 << 25),
        "T": _env_int("AHV_STORE_MAX_STEPS", 1 << 26),
        "B": _env_int("AHV_STORE_MAX_PAYLOAD", 1 << 37),
    }


_KIND = {"S": 0, "G": 1, "T": 2, "E": 3, "D": 4, "V": 5}  # csrc/include/ahv/store.h RowKind
_EXT_OF = {"S": ("S", "S4", "S8", "SP"), "D": ("D", "D8"), "E": ("E",), "V": ("V",), "G": ("G",), "T": ("T",)}
_FILL_NEG = ("v_head", "v_tail", "s_dlast", "d_prev", "e_next", "d_sess", "e_vsess", "t_saga", "d_hole")
_FILL_FREE = ("s_state", "g_state", "t_state")  # kFree8


def _fill(name: str) -> int:
    return -1 if name in _FILL_NEG else (255 if name in _FILL_FREE else 0)


def _extents(c: dict) -> dict:
    return {
        "S": c["S"], "S4": c["S"] * 4, "S8": c["S"] * 8, "SP": c["S"] * c["P"],
        "D": c["D"], "D8": c["D"] * 8, "E": c["E"], "V": c["V"], "G": c["G"], "T": c["T"], "SCR": c["X"],
    }


class StoreError(RuntimeError):
    """A store command failed for a reason the API layer does not map to a user error."""


class GovernanceStore:
    """Device tables + command transport + host-side allocators/interners.

    Row lifecycle: every session / saga / step / vouch-edge / delta row is handed
    out by a host allocator and is *live* while an API object refers to it (the
    view objects of :mod:`hypervisor._device` own their rows; dropping the last
    reference queues the row in ``_pending`` from ``__del__``).  Queued rows are
    reclaimed in batches: one ``OP_FREE_ROWS`` command marks them free on the
    device (after the hash engine has drained), then they return to the free
    list.  Creates on the device refuse a row that is not free, so a live row is
    never overwritten.  A full table grows (capacity doubles, rows keep their
    index) up to ``AHV_STORE_MAX_*``, then allocation raises :class:`StoreError`.
    """

    RECLAIM_BATCH = 4096  # released delta rows per reclaim (native: py_store.cpp kReclaimDeltas)
    # Command ring slots (512 B each, fine-grained device memory; AHV_STORE_SLOTS): a
    # post finding its slot still unexecuted spins until the worker catches up
    RING_SLOTS = 32768

    def __init__(self, device: str = "cuda", caps: Optional[dict] = None, idle_us: Optional[int] = None,
                 max_caps: Optional[dict] = None) -> None:
        dev = torch.device(device)
        if dev.type == "cuda":
            if not torch.cuda.is_available():
                raise RuntimeError("GovernanceStore(device='cuda') needs a HIP device")
            if dev.index is None:
                dev = torch.device("cuda", torch.cuda.current_device())
        elif dev.type != "cpu":
            raise ValueError(f"unsupported store device {dev}")
        self.device = dev
        self.caps = dict(default_caps(), **(caps or {}))
        self.max_caps = dict(default_max_caps(), **(max_caps or {}))
        for k, v in self.caps.items():
            if k in self.max_caps and self.max_caps[k] < v:
                self.max_caps[k] = v
        c = self.caps
        ext = _extents(c)
        self.tables: dict[str, torch.Tensor] = {}
        for name, ctype, kind in C.STORE_COLUMNS:
            self.tables[name] = torch.full((ext[kind],), _fill(name), dtype=_DTYPES[ctype], device=dev)
        if dev.type == "cuda":
            torch.cuda.synchronize(dev)
        ptrs = {k: v.data_ptr() for k, v in self.tables.items()}
        self._c = C.Store(
            dev.index if dev.type == "cuda" else -1, ptrs, dict(c),
            nslots=_env_int("AHV_STORE_SLOTS", self.RING_SLOTS),
            idle_us=idle_us if idle_us is not None else _env_int("AHV_STORE_IDLE_US", 500),
        )
        self._lock = threading.RLock()
        self._closed = False
        self.agents = Interner()  # DID → dense agent id
        self.pool = Interner()  # strings the batched pipeline renders (DIDs, change fields)
        # row allocators live in the native store (Store.alloc_row / release_row / reclaim_pool)
        self._alloc_row = self._c.alloc_row
        self._release_row = self._c.release_row
        self._tenant_v: dict[int, dict[str, int]] = {}  # tenant → liability session id → V row
        self._tenants = 0
        self.grows = {k: 0 for k in ("S", "G", "T", "E", "V", "D", "B")}
        self._waiters: list = []  # (seq, nres, future) of suspended asyncio calls
        self._polling = False
        self._deferred: list = []  # (seq, nres, check) of speculative posts not verified yet
        self.seed = int.from_bytes(os.urandom(8), "little") >> 1
        self._stamp_seq = 0
        self._id_ctr = 0  # device id generator counters handed out (reserve_ids)

    # -- allocation ----------------------------------------------------------
    def alloc(self, kind: str) -> int:
        """A free row of table ``kind`` (S sessions, E vouch edges, G sagas, T steps,
        V liability sessions): reclaimed rows first, then fresh ones; a full table
        grows (rows keep their index) up to its ``AHV_STORE_MAX_*`` ceiling."""
        k = _KIND[kind]
        r = self._alloc_row(k)
        while r < 0:
            self._grow(kind)
            r = self._alloc_row(k)
        return r

    def alloc_many(self, kind: str, n: int) -> np.ndarray:
        """``n`` free rows of table ``kind`` as int32 (reclaimed rows first, then fresh
        ones; the table grows as needed)."""
        if n <= 0:
            return np.zeros(0, dtype=np.int32)
        k = _KIND[kind]
        out = self._c.alloc_rows(k, n)
        while out is None:
            self._grow(kind)
            out = self._c.alloc_rows(k, n)
        return out

    def reserve_deltas(self, caps: list) -> tuple:
        """Delta rows + arena reservations of ``caps`` bytes each (batched pipeline):
        ``(rows int32 bytes, offsets int64 bytes)``."""
        raw = np.ascontiguousarray(caps, dtype="<i4").tobytes()
        tries = 0
        while True:
            r = self._c.reserve_deltas(raw)
            if r[1] is not None:
                return r
            self._make_room(r[0], tries)
            tries += 1

    def release(self, kind: str, row: int) -> None:
        """Queue a row whose last API reference is gone (safe to call from ``__del__``)."""
        self._release_row(_KIND[kind], row)

    def release_many(self, kind: str, rows) -> None:
        """Queue many rows: an int sequence or an int32 array (one native call)."""
        if type(rows) is list:
            if len(rows) <= 64:
                self._c.release_list(_KIND[kind], rows)
                return
        if len(rows):
            self._c.release_rows(_KIND[kind], np.ascontiguousarray(rows, dtype=np.int32))

    def _npend(self, kind: str) -> int:
        return self._c.npend(_KIND[kind])

    def reclaim(self, kind: Optional[str] = None) -> int:
        """Return queued rows to the free lists (one OP_FREE_ROWS per table); returns the count."""
        if self._closed:
            return 0
        total = 0
        with self._lock:
            for k in ([kind] if kind else list(_KIND)):
                total += self._c.reclaim_pool(_KIND[k])
        return total

    def live_rows(self) -> dict:
        """Rows held by API objects (allocated, not released), per table."""
        return {k: self._c.live_rows(v) for k, v in _KIND.items()}

    def _grow(self, kind: str) -> None:
        """Double table ``kind`` (rows keep their indices), up to its ``AHV_STORE_MAX_*``."""
        cur, mx = self.caps[kind], self.max_caps[kind]
        if cur >= mx:
            raise StoreError(
                f"store table {kind} full ({cur} live rows; ceiling AHV_STORE_MAX_* = {mx}): "
                "refusing to reuse live rows")
        new = min(mx, 2 * cur)
        with self._lock:
            self.drain()
            self._c.quiesce()
            caps = dict(self.caps, **{kind: new})
            ext = _extents(caps)
            grown = set(_EXT_OF[kind])
            P = self.caps["P"]
            for name, ctype, ek in C.STORE_COLUMNS:
                if ek not in grown:
                    continue
                old = self.tables[name]
                t = torch.full((ext[ek],), _fill(name), dtype=old.dtype, device=self.device)
                if ek == "SP":  # participant-major [P][S]: each participant plane keeps its rows
                    t.view(P, new)[:, :cur].copy_(old.view(P, cur))
                else:
                    t[: old.numel()].copy_(old)
                self.tables[name] = t
            if self.device.type == "cuda":
                torch.cuda.synchronize(self.device)
            self.caps = caps
            self._c.rebind({k: v.data_ptr() for k, v in self.tables.items()}, dict(caps))
            self.grows[kind] += 1

    def _grow_payload(self) -> None:
        cur, mx = self._c.payload_cap, self.max_caps["B"]
        if cur >= mx:
            raise StoreError(f"audit payload arena full ({cur} bytes; ceiling AHV_STORE_MAX_PAYLOAD)")
        with self._lock:
            self.drain()
            self._c.grow_payload(min(mx, 2 * cur))
            self.caps["B"] = self._c.payload_cap
            self.grows["B"] += 1

    def _make_room(self, code: int, tries: int) -> None:
        """capture / restore_delta reported a full table (-2 deltas, -3 arena)."""
        if tries == 0 and self.reclaim("D"):
            return
        if code == -2:
            self._grow("D")
        else:
            self._grow_payload()

    def new_tenant(self) -> int:
        self._tenants += 1
        return self._tenants

    def release_tenant(self, tenant: int, edges) -> None:
        """A vouching engine is gone: its edge rows and liability-session rows are reclaimable."""
        if edges:
            self.release_many("E", list(edges))
        vs = self._tenant_v.pop(tenant, None)
        if vs:
            self.release_many("V", list(vs.values()))

    def reserve_ids(self, n: int) -> int:
        """A range of ``n`` counters of the store's device id generator
        (``uuid4_words(seed, counter)``, batched pipelines); returns its base."""
        b = self._id_ctr
        self._id_ctr = b + n
        return b

    def next_stamp(self) -> int:
        """A creation stamp for a session whose id is not a uuid: a per-store serial
        with the top two bits 11.  A uuid4's low half always carries the RFC 4122
        variant bits 10 there, so no uuid session can share a stamp with one of
        these; the word is never zero (the serial starts at 1)."""
        self._stamp_seq += 1
        return (3 << 62) | (self._stamp_seq & ((1 << 62) - 1))

    def agent_id(self, did: str) -> int:
        return self.agents.intern(did)

    def did(self, agent_id: int) -> str:
        return self.agents.str(agent_id)

    def liability_id(self, tenant: int, session_id: str) -> int:
        d = self._tenant_v.get(tenant)
        if d is None:
            d = self._tenant_v[tenant] = {}
        v = d.get(session_id)
        if v is None:
            v = d[session_id] = self.alloc("V")
        return v

    def liability_lookup(self, tenant: int, session_id: str) -> int:
        d = self._tenant_v.get(tenant)
        return -1 if d is None else d.get(session_id, -1)

    # -- transport -----------------------------------------------------------
    def post(self, op: int, args: list, inline: Optional[bytes] = None, keep: bool = False) -> int:
        """Post a command; ``keep``: its results survive the recycling of its result
        slot until they are read (for results awaited after other sessions' posts)."""
        q = self._c.post(op, args, inline)
        if keep:
            self._c.keep(q)
        return q

    # -- speculation: commands whose outcome the host already knows -------------
    DEFERRED_MAX = 512  # unverified speculative posts before a blocking verification

    def post_checked(self, op: int, args: list, nres: int, check, inline: Optional[bytes] = None,
                     owner=None) -> int:
        """Post a command whose result the caller has predicted (from the same
        semantics.h predicates over state only it mutates) without waiting for it;
        ``check(result)`` returns None when the device agreed, else the exception
        the prediction's owner gets.  Results are verified by :meth:`verify_deferred`
        (before every later store call and whenever the list grows long).

        ``owner``: the API object the prediction belongs to (a device session).  A
        disagreement — an internal invariant violation — is handed to it
        (``owner._spec_failed(exc)``) and raised on *its* next operation; it never
        surfaces in a call made by another session or tenant sharing the store."""
        q = self._c.post(op, args, inline)
        self._c.keep(q)
        self.defer(q, nres, check, owner)
        return q

    def post_expect(self, op: int, args: list, want: tuple, token: tuple, inline: Optional[bytes] = None) -> int:
        """The fast form of :meth:`post_checked`: the prediction is the leading result
        words ``want`` (None = any value), checked natively in post order; a mismatch
        hands ``token`` = (owner, make_error, arg) to :meth:`verify_deferred`, which
        raises ``make_error(arg, result)`` in the owner's next call (or here, unowned)."""
        return self._c.post_expect(op, args, inline, want, token)

    def expect(self, seq: int, want: tuple, token: tuple) -> None:
        """:meth:`post_expect` for a command already posted."""
        self._c.expect(seq, want, token)

    def pending_checks(self) -> int:
        """Speculated posts not verified yet."""
        return len(self._deferred) + self._c.n_expects()

    def defer(self, seq: int, nres: int, check, owner=None) -> None:
        """Verify a kept post (``post(..., keep=True)``) later instead of awaiting it."""
        self._deferred.append((seq, nres, check, owner))
        if len(self._deferred) >= self.DEFERRED_MAX:
            self.verify_deferred(block=True)

    def verify_deferred(self, block: bool = False) -> None:
        """Check speculatively posted commands whose results are in (all of them with
        ``block``).  A disagreement goes to the prediction's owner; only an
        unowned prediction raises here."""
        if block:
            self._c.check_frees(True)  # row reclaims posted without waiting (native allocator)
        bad = self._c.verify_expects(block)
        err = self._distribute(bad) if bad is not None else None
        ds = self._deferred
        if not ds:
            if err is not None:
                raise err
            return
        self._deferred = []
        pending, misses = [], 0
        try_result = self._c.try_result
        for i, d in enumerate(ds):
            r = try_result(d[0], d[1], 1_000_000_000 if block else 0)
            if r is None:
                pending.append(d)
                misses += 1
                if misses >= self.POLL_MISSES:  # results complete in post order: the rest are pending too
                    pending.extend(ds[i + 1:])
                    break
                continue
            misses = 0
            e = d[2](r)
            if e is None:
                continue
            if d[3] is not None:
                d[3]._spec_failed(e)
            elif err is None:
                err = e
        self._deferred = pending + self._deferred
        if err is not None:
            raise err

    @staticmethod
    def _distribute(bad) -> Optional[Exception]:
        """Hand each mismatched expectation ``((owner, make_error, arg), result)`` to
        its owner; returns the first unowned error (the caller raises it)."""
        err = None
        for (owner, make, arg), r in bad:
            e = make(arg, r)
            if owner is not None:
                owner._spec_failed(e)
            elif err is None:
                err = e
        return err

    def discard(self, seq: int) -> None:
        """Forget a kept result (``post(..., keep=True)``) that will never be read."""
        self._c.discard(seq)

    def call(self, op: int, args: list, nres: int = 4, inline: Optional[bytes] = None) -> tuple:
        self.verify_deferred()
        return self._c.call(op, args, nres, inline)

    def result(self, seq: int, nres: int = 4) -> tuple:
        return self._c.result(seq, nres)

    def stage(self, data: bytes) -> int:
        return self._c.stage(data)

    def bulk(self, off: int, n: int) -> bytes:
        return self._c.bulk(off, n)

    def payload(self, off: int, n: int) -> bytes:
        return self._c.payload(off, n)

    def capture(self, slot: int, turn: int, ts_us: int, delta, parent: Optional[str] = None) -> tuple:
        """(delta row, arena offset, length, sequence, predicted digest): the last is
        the device's digest computed on the host (``parent``: the previous capture's
        predicted digest; None for turn 1 or when unknown → no prediction)."""
        r = self._c.capture(slot, turn, ts_us, delta, parent)  # reclaims released delta rows natively
        tries = 0
        while r[0] <= -2:
            self._make_room(r[0], tries)
            tries += 1
            r = self._c.capture(slot, turn, ts_us, delta, parent)
        return r

    def capture_bytes(self, slot: int, turn: int, ts_us: int, raw: bytes, null_at: int,
                      parent: Optional[str] = None) -> tuple:
        r = self._c.capture_bytes(slot, turn, ts_us, raw, null_at, parent)
        tries = 0
        while r[0] <= -2:
            self._make_room(r[0], tries)
            tries += 1
            r = self._c.capture_bytes(slot, turn, ts_us, raw, null_at, parent)
        return r

    def restore_delta(self, data: bytes) -> tuple:
        """(delta row, arena offset) for a checkpointed record."""
        r = self._c.restore_delta(data)
        tries = 0
        while r[0] <= -2:
            self._make_room(r[0], tries)
            tries += 1
            r = self._c.restore_delta(data)
        return r

    # -- asyncio API -------------------------------------------------------------
    SPIN_NS = 150_000  # spin this long for a result when the event loop has nothing else to run
    # ... and this long when other tasks are ready: a suspension + wake-up costs more
    # CPU than a short spin when the round trip is a few µs (AHV_STORE_SPIN_BUSY_NS)
    SPIN_BUSY_NS = _env_int("AHV_STORE_SPIN_BUSY_NS", 15_000)

    async def result_async(self, seq: int, nres: int = 4, spin_busy: Optional[int] = None) -> tuple:
        """The results of ``seq`` without blocking the event loop: when other tasks
        are ready (many sessions in flight) the caller suspends at once and a
        loop-driven poller resumes it; otherwise it spins briefly first (a lone
        pipeline's round trip is a few µs, cheaper than a suspension)."""
        import asyncio

        loop = asyncio.get_running_loop()
        ready = getattr(loop, "_ready", None)
        spin = (self.SPIN_BUSY_NS if spin_busy is None else spin_busy) if ready else self.SPIN_NS
        r = self._c.try_result(seq, nres, spin)
        if r is not None:
            return r
        fut = loop.create_future()
        self._waiters.append((seq, nres, fut))
        if not self._polling:
            self._polling = True
            loop.call_soon(self._poll, loop)
        return await fut

    POLL_MISSES = 16  # consecutive pending waiters after which a poll pass stops scanning

    def _poll(self, loop) -> None:
        """Deliver completed results to their waiters.  Waiters are in post (= seq)
        order and the worker completes commands in order (only deferred captures
        finish after later commands), so a pass stops after ``POLL_MISSES``
        consecutive pending ones: with thousands of sessions in flight a pass costs
        O(completed), not O(waiting)."""
        ws = self._waiters
        self._waiters = []
        keep = []
        misses = 0
        try_result = self._c.try_result
        for i, w in enumerate(ws):
            try:
                r = try_result(w[0], w[1], 0)
            except Exception as e:  # noqa: BLE001 - delivered to the awaiting call
                if not w[2].done():
                    w[2].set_exception(e)
                continue
            if r is None:
                keep.append(w)
                misses += 1
                if misses >= self.POLL_MISSES:
                    keep.extend(ws[i + 1:])
                    break
            else:
                misses = 0
                if not w[2].done():
                    w[2].set_result(r)
        if self._waiters:
            keep.extend(self._waiters)
        self._waiters = keep
        if keep:
            loop.call_soon(self._poll, loop)
        else:
            self._polling = False

    async def call_async(self, op: int, args: list, nres: int = 4, inline: Optional[bytes] = None,
                         spin_busy: Optional[int] = None) -> tuple:
        """Post and await.  ``spin_busy``: how long to spin for the result while other
        tasks are ready (default SPIN_BUSY_NS); 0 for commands that wait for the hash
        engine (a terminate's root), whose answer is tens of µs away."""
        self.verify_deferred()
        return await self.result_async(self._c.post(op, args, inline), nres, spin_busy)

    def drain(self) -> None:
        self._c.drain()

    def flush(self) -> None:
        """Make every table write visible to other kernels / torch reads (release)."""
        self.call(OP_FLUSH, [], 1)

    def acquire(self) -> None:
        """Make rows written by other kernels (batched pipeline) visible to the worker."""
        self.call(OP_ACQUIRE, [], 1)

    def close(self) -> None:
        self._closed = True
        self._c.close()

    @property
    def is_gpu(self) -> bool:
        return self._c.gpu

    def info(self) -> dict:
        d = dict(self._c.info())
        d["live_rows"] = self.live_rows()
        d["caps"] = dict(self.caps)
        d["grows"] = dict(self.grows)
        return d

    def write_rows(self, rows: dict) -> None:
        """Scatter host values into table rows: ``{column: (indices, values)}``.

        Used by checkpoint restore and by host-side bulk loads.  The worker's
        dirty lines are written back first (release) and it re-reads the rows
        afterwards (acquire), so the tensor writes and the command stream agree.
        """
        self.drain()
        cuda = self.device.type == "cuda"
        if cuda:
            self.flush()
        for col, (idx, vals) in rows.items():
            if not len(idx):
                continue
            last = dict(zip(idx, vals))  # a later write to the same row wins (deterministically)
            idx, vals = list(last.keys()), list(last.values())
            t = self.tables[col]
            if t.dtype == torch.int32:
                vals = [v - (1 << 32) if v >= 1 << 31 else v for v in vals]
            t[torch.tensor(idx, dtype=torch.int64, device=self.device)] = torch.tensor(vals, dtype=t.dtype).to(
                self.device)
        if cuda:
            torch.cuda.synchronize(self.device)
            self.acquire()

    def write_columns(self, cols: dict) -> None:
        """Vectorized :meth:`write_rows`: ``{column: (int64 element indices, values)}``
        with numpy / torch arrays (one ``index_copy_`` per column; indices must be
        distinct).  Checkpoint restore writes whole tables this way."""
        self.drain()
        cuda = self.device.type == "cuda"
        if cuda:
            self.flush()
        for col, (idx, vals) in cols.items():
            if len(idx) == 0:
                continue
            t = self.tables[col]
            ix = torch.as_tensor(np.ascontiguousarray(idx, dtype=np.int64)).to(self.device)
            if isinstance(vals, torch.Tensor):  # device-resident values (migration): no host copy
                v = vals.reshape(-1)
                if v.dtype != t.dtype:  # same-width integers are bit patterns (uint32 words)
                    v = v.view(t.dtype) if v.element_size() == t.element_size() and not v.is_floating_point() \
                        and not t.is_floating_point() else v.to(t.dtype)
                t.index_copy_(0, ix, v.to(self.device))
                continue
            want = _NP_OF[t.dtype]
            a = np.ascontiguousarray(vals)
            if a.dtype != want:  # same-width integers are bit patterns (uint32 words); else convert
                same = a.dtype.itemsize == want.itemsize and a.dtype.kind in "iu" and want.kind in "iu"
                a = a.view(want) if same else a.astype(want)
            t.index_copy_(0, ix, torch.from_numpy(a).to(self.device))
        if cuda:
            torch.cuda.synchronize(self.device)
            self.acquire()

    def column(self, name: str) -> torch.Tensor:
        """A table column as the worker last wrote it (flushes pending device writes
        first).  Growth replaces the tensors: fetch a column again after creating rows."""
        self.drain()
        if self.device.type == "cuda":
            self.flush()
        return self.tables[name]

    # -- batched reads ----------------------------------------------------------
    def read_sessions(self, slots, parts: bool = False):
        """Header rows (and participant rows) of many sessions, O(1) commands:
        ``(hdr uint64[n, STORE_HDR_WORDS], parts uint64[n, P, 5] | None)``.  Header
        layout: ``exec_read_many`` in ``csrc/include/ahv/store.h``."""
        import numpy as np

        slots = list(slots)
        n = len(slots)
        H = C.STORE_HDR_WORDS
        P = self.caps["P"]
        per = 8 * H + (40 * P if parts else 0)
        chunk = max(1, min(self._c.bulk_cap // per, self._c.staging_cap // 8))
        hdr = np.zeros((n, H), dtype=np.uint64)
        prt = np.zeros((n, P, 5), dtype=np.uint64) if parts else None
        for i in range(0, n, chunk):
            part = slots[i: i + chunk]
            k = len(part)
            cnt, off, inl = self.index_args(part)
            r = self.call(OP_SESS_READ_MANY, [cnt, off, 0, int(parts)], 1, inl)
            if r[0]:
                raise StoreError(f"OP_SESS_READ_MANY failed with status {r[0]}")
            raw = self.bulk(0, 8 * H * k + (40 * P * k if parts else 0))
            words = np.frombuffer(raw, dtype=np.uint64)
            hdr[i: i + k] = words[: H * k].reshape(k, H)
            if parts:
                prt[i: i + k] = words[H * k:].reshape(k, P, 5)
        return hdr, prt

    def gather(self, cols: dict) -> dict:
        """``{column: row indices}`` → ``{column: numpy array}``: a device gather of
        every requested column after one release of the worker's writes (O(1)
        store commands however many rows)."""
        import numpy as np

        if not any(len(v) for v in cols.values()):
            return {k: np.zeros(0, dtype=np.int64) for k in cols}
        self.drain()
        if self.device.type == "cuda":
            self.flush()
        out = {}
        for name, idx in cols.items():
            t = self.tables[name]
            ix = torch.from_numpy(np.asarray(idx, dtype=np.int64)).to(self.device)
            out[name] = t.index_select(0, ix).cpu().numpy()
        return out

    # -- index lists -----------------------------------------------------------
    def index_args(self, idx: list) -> tuple:
        """(count, staging offset, inline bytes) for an int32 index list argument."""
        n = len(idx)
        raw = struct.pack(f"<{n}i", *idx)
        if n <= 96:
            return n, 0, raw
        return n, self.stage(raw), None


_STORES: dict = {}
_STORES_LOCK = threading.Lock()


def shared_store(device: str) -> GovernanceStore:
    """The process-wide store of ``device`` (created on first use)."""
    key = str(torch.device(device))
    st = _STORES.get(key)
    if st is None:
        with _STORES_LOCK:
            st = _STORES.get(key)
            if st is None:
                st = GovernanceStore(device)
                _STORES[key] = st
    return st


@atexit.register
def _close_all() -> None:
    for st in list(_STORES.values()):
        try:
            st.close()
        except Exception:
            pass
