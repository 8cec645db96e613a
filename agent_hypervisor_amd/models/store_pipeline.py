"""Batched, heterogeneous governance pipelines written straight into the store.

:meth:`hypervisor.Hypervisor.run_pipelines` runs the reference pipeline
(``benchmarks/bench_hypervisor.py:217-239``) for many sessions in three gfx950
launches over the *store's* tables (``csrc/hip/store_pipeline.hip``) plus the K09
root kernel — and the sessions it creates are ordinary device sessions of the
public API: ``hv.get_session(sid)`` returns a ``ManagedSession`` whose views read
the same rows, ``verify_audit`` / ``terminate_session`` / snapshots work on them,
and their rows are reclaimed like any other once unreferenced.

Heterogeneity (:class:`PipelineSpec`, one per session or one shared): any number
of joins with per-agent σ (ring gate + admission in order — reference
``core.py:106-185``), per-delta agents and change lists, saga steps with
pre-resolved outcomes — ``failures`` attempts fail before one succeeds; with more
failures than ``1 + max_retries`` attempts the step fails and the saga stops —
and reverse-order compensation (``saga/orchestrator.py:77-198``).  Executors are
not run: the outcomes are inputs (a batch replays decided work at device speed).

Sessions are registered lazily: the hypervisor holds a small placeholder per
session and builds the Python views only when one is first used, so a batch of
10⁵ sessions costs a few µs of host work per session, not a view graph each.
"""

from __future__ import annotations

from dataclasses import dataclass, field
from typing import Optional, Sequence

import numpy as np
import torch

from agent_hypervisor_amd._native import C

REFERENCE_JOINS = (("did:mesh:a", 0.8),)
REFERENCE_DELTAS = tuple(("did:mesh:a", ((f"/f{i}", "add", f"h{i}"),)) for i in range(3))
REFERENCE_STEPS = (("action", "did:mesh:a", "/api/action", None, 0, 0),)

# A/B switches of the batch kernels' work layout (AHV_SP_ORDER bit0 chain lanes by work, bit1
# render lanes by record shape with co-located arena space, bit2 K09 lanes by chain length;
# AHV_SP_PREFIX: where the records' parent-independent SHA blocks are compressed)
import os as _os  # noqa: E402

_SP_ORDER = int(_os.environ.get("AHV_SP_ORDER", "5"))
# render | kernel | sorted (its own kernel, lanes grouped by SHA work) | chain (no split: the chain lane hashes all)
_SP_PREFIX = _os.environ.get("AHV_SP_PREFIX", "sorted")
_SP_PREFIX_IN_RENDER = 0 if _SP_PREFIX in ("kernel", "sorted") else 1
# record heads rendered once per distinct (agent, changes) of a batch and copied by
# the render kernel (C.frag_pack), AHV_SP_FRAGS=1.  Off by default: the kernel gains
# 18 µs per 10^6 sessions (render 707 -> 689 µs, profiles/r6/hetero_frags_r6s.jsonl)
# but the host pass costs ≈ 0.4 µs per delta in prepare, which the public API times
_SP_FRAGS = _os.environ.get("AHV_SP_FRAGS", "0") != "0"
# the rows pass's blocks share one launch with the render pass's (both wait on memory
# most of the time: store_pipe_render_rows_kernel), the prefix SHA pass on its own
# (render + rows 775 µs, prefix 486 per 10^6 sessions: 1.91 vs 1.95 ms per step,
# profiles/r6/hetero_rows_layout_ab_r6an.txt); AHV_SP_OVERLAP=1: the rows blocks share
# the prefix pass's launch instead (store_pipe_prefix_rows_kernel); 0: rows, render,
# prefix as three passes
_SP_OVERLAP = int(_os.environ.get("AHV_SP_OVERLAP", "2"))
# the committed chains' Merkle roots (K09) folded in the chain kernel's lanes as the
# digests are produced; AHV_SP_CHAIN_ROOTS=0: the K09 kernel afterwards (_k09_plan)
_SP_CHAIN_ROOTS = _os.environ.get("AHV_SP_CHAIN_ROOTS", "1") != "0" and _SP_PREFIX != "chain"

_STATUS = {0: "ok", 1: "row_in_use", 2: "join_refused", 3: "activate_refused", 4: "step_failed",
           5: "terminate_refused", 6: "record_overflow"}


@dataclass(frozen=True)
class PipelineSpec:
    """One session's pipeline.

    ``joins``: ``(agent_did, sigma_raw)`` in order.  ``deltas``: ``(agent_did,
    changes)`` with changes ``(path, operation, content_hash[, previous_hash])``.
    ``steps``: ``(action_id, agent_did, execute_api, undo_api, max_retries,
    failures)``.  ``config``: a :class:`hypervisor.SessionConfig` (default one)."""

    joins: Sequence[tuple] = REFERENCE_JOINS
    deltas: Sequence[tuple] = REFERENCE_DELTAS
    steps: Sequence[tuple] = REFERENCE_STEPS
    activate: bool = True
    terminate: bool = True
    compensate: bool = True
    config: Optional[object] = None
    creator_did: str = "did:mesh:admin"


@dataclass
class PipelineRun:
    """What one :meth:`Hypervisor.run_pipelines` call produced."""

    session_ids: list
    status: np.ndarray        # per session, 0 = every stage admitted (see status_name)
    join_rings: np.ndarray    # per join, in spec order
    join_codes: np.ndarray
    device_seconds: float = 0.0
    prepare_seconds: float = 0.0   # host packing + row allocation + argument upload
    finish_seconds: float = 0.0    # read-back + lazy registration
    _roots: tuple = field(default=(), repr=False)  # (committed session indices, their roots as one hex string)

    @property
    def roots(self) -> dict:
        """Session id → committed Merkle root (64 hex digits), built on first access."""
        r = self.__dict__.get("_roots_dict")
        if r is None:
            idx, flat = self._roots or ((), "")
            ids = self.session_ids
            r = self.__dict__["_roots_dict"] = {ids[i]: flat[64 * j:64 * j + 64]
                                                for j, i in enumerate(list(idx))}
        return r

    def status_name(self, i: int) -> str:
        return _STATUS.get(int(self.status[i]), str(int(self.status[i])))

    @property
    def ok(self) -> int:
        return int((self.status == 0).sum())


class _Batch:
    """Host metadata of one batch: what a lazy session needs to build its views.

    Row ownership: a session that builds its views hands its rows to them
    (``built``); the rows of sessions dropped unbuilt are returned in bulk — a
    dropped session only appends its index to ``dead`` and every ``_FLUSH`` of
    them (and whatever is left when the batch itself goes) are released with one
    vectorized gather per table."""

    __slots__ = ("store", "specs", "shared", "ids", "slots", "t0", "doff", "drows", "dlen", "dhash",
                 "delta_off", "gslots", "step_off", "tslots", "status", "built", "released", "dead",
                 "index", "views", "committed", "_saga_ids", "_step_ids", "id_seed", "gid_base", "tid_base",
                 "__weakref__")

    def reserve_saga_ids(self) -> None:
        """Give the batch's saga / step ids fixed counters of the store's id
        generator: ids are formatted only when first needed (uuid4 words of
        (seed, counter)), and a checkpoint that saves the counters restores the
        same ids whether or not they were formatted before."""
        st = self.store
        self.id_seed = st.seed
        self.gid_base = st.reserve_ids(len(self.gslots))
        self.tid_base = st.reserve_ids(int(self.step_off[-1]))

    def saga_ids(self) -> tuple:
        """(saga id per session or None, step id per step row): formatted once, in
        bulk, the first time a view or a summary needs them."""
        if self._saga_ids is None:
            has = self.gslots >= 0
            nt = int(self.step_off[-1])
            if getattr(self, "id_seed", None) is not None:
                allg = C.uuids_from_counters(self.id_seed, self.gid_base, len(self.gslots), "saga:")
                self._saga_ids = [g if h else None for g, h in zip(allg, has.tolist())]
                self._step_ids = C.uuids_from_counters(self.id_seed, self.tid_base, nt, "step:") if nt else []
            else:
                ng = int(has.sum())
                sg, _ = C.uuid4_many(ng, "saga:") if ng else ([], b"")
                it = iter(sg)
                self._saga_ids = [next(it) if h else None for h in has.tolist()]
                self._step_ids = C.uuid4_many(nt, "step:")[0] if nt else []
        return self._saga_ids, self._step_ids

    def saga_summaries(self, rows: dict, idx) -> list:
        """Summary dicts (Hypervisor.saga_summaries form) of the sagas of unbuilt
        sessions ``idx``, from gathered ``rows`` (g_* per saga, t_* per step)."""
        from hypervisor._clock import from_us
        from hypervisor.saga.state_machine import SagaState, StepState

        gids, tids = self.saga_ids()
        gst, sst = list(SagaState), list(StepState)
        out, gk, tk = [], 0, 0
        for i in idx:
            if self.gslots[i] < 0:
                continue
            sp = _spec(self, i)
            s0, s1 = int(self.step_off[i]), int(self.step_off[i + 1])
            steps = []
            for k in range(s0, s1):
                a = sp.steps[k - s0]
                t0, t1 = int(rows["t_started"][tk]), int(rows["t_completed"][tk])
                steps.append({"step_id": tids[k], "action_id": a[0], "agent_did": a[1],
                              "state": sst[int(rows["t_state"][tk]) & 0xFF].value,
                              "retry_count": int(rows["t_retry"][tk]), "error": None,
                              "started_at": from_us(t0) if t0 else None, "completed_at": from_us(t1) if t1 else None})
                tk += 1
            c1 = int(rows["g_completed"][gk])
            out.append({"saga_id": gids[i], "session_id": self.ids[i],
                        "state": gst[int(rows["g_state"][gk]) & 0xFF].value, "error": None,
                        "created_at": from_us(int(rows["g_created"][gk])),
                        "completed_at": from_us(c1) if c1 else None, "steps": steps})
            gk += 1
        return out

    def saga_row_slots(self, idx) -> tuple:
        """(saga rows, step rows) of the unbuilt sessions ``idx`` in summary order."""
        gi, ti = [], []
        for i in idx:
            g = int(self.gslots[i])
            if g >= 0:
                gi.append(g)
                ti.extend(self.tslots[int(self.step_off[i]):int(self.step_off[i + 1])].tolist())
        return gi, ti

    _FLUSH = 8192

    # -- the session table's view of the batch (hypervisor.session.table) --------
    def view(self, i: int):
        """The ManagedSession of session ``i`` (built on first use; it then owns the rows)."""
        m = self.views.get(i)
        if m is None:
            from hypervisor.core import ManagedSession

            m = self.views[i] = ManagedSession(*materialize(self, i))
            self.built[i] = True
        return m

    def forget(self, i: int):
        """Session ``i`` left the hypervisor: its view (if built) or its rows go."""
        m = self.views.pop(i, None)
        if m is None:
            self.drop(i)
        return m

    def entries(self):
        from hypervisor.core import LazyManagedSession

        views = self.views
        for i in self.index.values():
            m = views.get(i)
            yield m if m is not None else LazyManagedSession(self, i)

    def rowref(self, i: int):
        m = self.views.get(i)
        if m is not None:
            return m.sso
        return _RowRef(int(self.slots[i]), self.ids[i], _spec(self, i).creator_did)

    def rows(self, committed: bool = False) -> tuple:
        """(slots, session ids, creator DIDs) of the batch's sessions (or of its
        committed ones) in order — what a batched snapshot read needs."""
        idx = np.fromiter(self.index.values(), dtype=np.int64, count=len(self.index))
        if committed:
            idx = idx[self.committed[idx]]
        ids = self.ids
        if self.shared:
            creators = [self.specs.creator_did] * len(idx)
        else:
            creators = [self.specs[i].creator_did for i in idx.tolist()]
        return self.slots[idx], [ids[i] for i in idx.tolist()], creators

    def drop(self, i: int) -> None:
        self.dead.append(i)
        if len(self.dead) >= self._FLUSH:
            self.release(np.asarray(self.dead, dtype=np.int64))
            self.dead = []

    def release(self, idx: np.ndarray) -> None:
        """Return the rows of unbuilt sessions ``idx`` to the store (once each)."""
        idx = idx[~self.built[idx] & ~self.released[idx]]
        if not len(idx):
            return
        self.released[idx] = True
        st = self.store
        n = len(self.slots)
        sel = np.zeros(n, dtype=bool)
        sel[idx] = True
        refused = self.status == 1  # the device kept the row from us: not ours to free
        st.release_many("S", self.slots[sel & ~refused])
        nd = np.diff(self.delta_off)
        if nd.any():
            st.release_many("D", self.drows[np.repeat(sel, nd)])
        g = self.gslots[sel]
        g = g[g >= 0]
        if len(g):
            st.release_many("G", g)
            st.release_many("T", self.tslots[np.repeat(sel, np.diff(self.step_off))])

    def __del__(self) -> None:
        try:
            self.release(np.arange(len(self.slots), dtype=np.int64))
        except Exception:  # noqa: BLE001 - interpreter shutdown
            pass


def mixed_specs(n: int, seed: int = 5, distinct: int = 4096, agents: int = 64, prefix: str = "did:mesh:m") -> list:
    """``n`` heterogeneous pipelines (a pool of ``distinct`` random specs, dealt
    out in a seeded order): 1–5 joins with per-agent σ (some refused by the gate
    or by capacity), 0–4 audit deltas of 0–3 changes by varying agents, 0–3 saga
    steps with retries, failures and compensation, varied configs, and sessions
    that never activate or terminate.  The mix ``bench.py --mix hetero`` times."""
    import random

    from hypervisor.models import SessionConfig

    rng = random.Random(seed)
    dids = [f"{prefix}{k}" for k in range(agents)]
    sigmas = [0.3, 0.55, 0.61, 0.7, 0.8, 0.96]
    pool = []
    for _ in range(distinct):
        joins = tuple((rng.choice(dids), rng.choice(sigmas + [rng.random()])) for _ in range(rng.randint(1, 5)))
        deltas = tuple((rng.choice(dids), tuple((f"/p{rng.randrange(50)}", rng.choice(["add", "update", "delete"]),
                                                 rng.choice([None, f"h{rng.randrange(1000)}"]))
                                                for _ in range(rng.randrange(0, 4))))
                       for _ in range(rng.randrange(0, 5)))
        steps = tuple((f"act{k}", rng.choice(dids), f"/api/{k}", rng.choice([None, f"/undo/{k}"]),
                       rng.randrange(0, 3), rng.choice([0, 0, 0, 1, 2, 5])) for k in range(rng.randrange(0, 4)))
        cfg = SessionConfig(max_participants=rng.choice([2, 3, 10]), min_sigma_eff=rng.choice([0.5, 0.6, 0.9]),
                            enable_audit=rng.random() < 0.9)
        pool.append(PipelineSpec(joins=joins, deltas=deltas, steps=steps, activate=rng.random() < 0.95,
                                 terminate=rng.random() < 0.9, compensate=rng.random() < 0.7, config=cfg,
                                 creator_did=rng.choice(dids)))
    order = np.random.default_rng(seed).integers(0, distinct, size=n)
    return [pool[i] for i in order.tolist()]


def _spec(b: _Batch, i: int) -> PipelineSpec:
    return b.specs if b.shared else b.specs[i]


def _escaped_len(pool, cache: dict, s: Optional[str]) -> int:
    if s is None:
        return 4
    n = cache.get(s)
    if n is None:
        n = cache[s] = len(pool.escaped(pool.intern(s))) + 2
    return n


_FIXED = 14 + 14 + 16 + 7 + 1 + 17 + 16 + 46 + 15 + 34 + 13 + 1  # literals, session id, timestamp


def _delta_cap(pool, cache, did: str, changes, turn: int) -> int:
    n = _FIXED + 2 * len(str(turn)) + (66 if turn > 1 else 4) + _escaped_len(pool, cache, did)
    for k, c in enumerate(changes):
        n += 17 + 15 + 10 + 19 + 1 + (2 if k else 0)
        n += _escaped_len(pool, cache, c[2]) + _escaped_len(pool, cache, c[1]) + _escaped_len(pool, cache, c[0])
        n += _escaped_len(pool, cache, c[3] if len(c) > 3 else None)
    return (n + 8 + 63) & ~63


class _CfgHolder:
    """A spec-shaped holder of one config (cfg_row caches by the config object)."""

    __slots__ = ("config",)

    def __init__(self, config) -> None:
        self.config = config


def run(hv, specs, n: Optional[int] = None) -> PipelineRun:
    """Build the batch arrays, run the store pipeline, register lazy sessions."""
    import time

    t0 = time.perf_counter()
    p = prepare(hv, specs, n)
    t1 = time.perf_counter()
    launch(p)
    t2 = time.perf_counter()
    r = finish(hv, p)
    r.prepare_seconds, r.finish_seconds = t1 - t0, time.perf_counter() - t2
    return r


class Prepared:
    """A packed batch: its store rows (allocated), device argument arrays and the
    host-side metadata :func:`finish` needs.  :func:`launch` runs it; a benchmark
    may re-run the same batch after :meth:`reset` (the rows freed in place)."""

    def reset(self, all_rows: bool = False) -> None:
        """Free the batch's session rows in place (on the stream), so :func:`launch`
        can run the whole pipeline over them again.  Its saga and step rows stay
        allocated to it — the rows pass writes them whole without a free-row check —
        unless ``all_rows`` frees them too."""
        t = self.store.tables
        ixs = self.__dict__.get("_reset_ix")
        if ixs is None:  # int64 row indices, converted once
            ixs = self.__dict__["_reset_ix"] = [
                (col, ix.to(torch.int64)) for col, ix in (("s_state", self.tens["slot"]), ("g_state", self.g_live),
                                                          ("t_state", self.t_live)) if ix is not None and ix.numel()]
        for col, ix in (ixs if all_rows else ixs[:1]):
            t[col].index_fill_(0, ix, 255)  # kFree8
        self.tens["status"].zero_()  # the kernels write only codes other than ok over a zeroed array


def prepare(hv, specs, n: Optional[int] = None) -> "Prepared":
    """Pack ``specs`` into device arrays over freshly allocated store rows."""
    from hypervisor._clock import now_us
    from hypervisor.models import ConsistencyMode, SessionConfig

    st = hv._store
    if st is None:
        raise RuntimeError("run_pipelines needs a device-backed Hypervisor (device='cuda' or 'cpu')")
    shared = isinstance(specs, PipelineSpec)
    if shared:
        if n is None:
            raise ValueError("run_pipelines(spec) needs n")
    else:
        specs = list(specs)
        n = len(specs)
    dev = st.device
    pool = st.pool
    cache: dict = {}
    ids, words = C.uuid4_many(n, "session:")
    slots = np.asarray(st.alloc_many("S", n), dtype=np.int32)
    t0 = now_us()

    def per_session(fn, dtype):
        if shared:
            return np.full(n, fn(specs), dtype=dtype)
        return np.asarray([fn(s) for s in specs], dtype=dtype)

    def cfg(s):
        return s.config or SessionConfig()

    cfg_cache: dict = {}

    def cfg_row(s):  # (max_participants, min_sigma_eff, audit | strong) per distinct config object
        c = s.config
        r = cfg_cache.get(id(c))
        if r is None:
            cc = c or SessionConfig()
            r = cfg_cache[id(c)] = (int(cc.max_participants), float(cc.min_sigma_eff),
                                    (1 if cc.enable_audit else 0)
                                    | (2 if ConsistencyMode(cc.consistency_mode) is ConsistencyMode.STRONG else 0), c)
        return r

    if shared:
        creator = per_session(lambda s: st.agent_id(s.creator_did), np.int32)
        mp, ms, cf, _ = cfg_row(specs)
        maxpart = np.full(n, mp, dtype=np.int32)
        minsig = np.full(n, ms, dtype=np.float64)
        flags = np.full(n, cf | (4 if specs.activate else 0) | (8 if specs.terminate else 0)
                        | (16 if specs.compensate else 0), dtype=np.uint8)
        joins = list(specs.joins)
        j_agent = np.tile(np.asarray([st.agent_id(d) for d, _ in joins], dtype=np.int32), n)
        j_sigma = np.tile(np.asarray([float(x) for _, x in joins], dtype=np.float64), n)
        k = len(joins)
        join_off = np.arange(0, (n + 1) * k, k, dtype=np.int32) if k else np.zeros(n + 1, dtype=np.int32)
        deltas = list(specs.deltas)
        per = len(deltas)
        delta_off = np.arange(0, (n + 1) * per, per, dtype=np.int32) if per else np.zeros(n + 1, dtype=np.int32)
        d_pool = [pool.intern(did) for did, _ in deltas]
        ch_off, ch_rows = [0], []
        for did, chs in deltas:
            for c in chs:
                ch_rows.append([pool.intern(c[0]), pool.intern(c[1]),
                                pool.intern(c[2]) if c[2] is not None else -1,
                                pool.intern(c[3]) if len(c) > 3 and c[3] is not None else -1])
            ch_off.append(len(ch_rows))
        caps = np.tile(np.asarray([_delta_cap(pool, cache, did, chs, t + 1) for t, (did, chs) in enumerate(deltas)],
                                  dtype=np.int32), n)
        d_pool = np.tile(np.asarray(d_pool, dtype=np.int32), n)
        base = np.asarray(ch_off[:-1], dtype=np.int32)
        per_ch = ch_off[-1]
        ch_off_all = np.append(np.tile(base, n) + np.repeat(np.arange(n, dtype=np.int32) * per_ch, per), per_ch * n)
        ch_rows = np.tile(np.asarray(ch_rows or [[0, 0, 0, 0]], dtype=np.int32), (n, 1)) if ch_rows else []
        steps = list(specs.steps)
        ks = len(steps)
        step_off = np.arange(0, (n + 1) * ks, ks, dtype=np.int32) if ks else np.zeros(n + 1, dtype=np.int32)
        s_undo = np.tile(np.asarray([1 if x[3] else 0 for x in steps], dtype=np.uint8), n)
        s_retry = np.tile(np.asarray([int(x[4]) for x in steps], dtype=np.int32), n)
        s_fail = np.tile(np.asarray([min(255, int(x[5])) for x in steps], dtype=np.uint8), n)
    else:  # one spec per session: flattened natively (csrc/host/py_runtime.cpp pack_specs)
        packed = C.pack_specs(specs, st.agents._pool, pool._pool, lambda c: cfg_row(_CfgHolder(c))[:3], _FIXED)
        col = lambda k, dt: np.frombuffer(packed[k], dtype=dt)  # noqa: E731
        creator, maxpart, minsig, flags = col("creator", np.int32), col("maxpart", np.int32), \
            col("minsig", np.float64), col("flags", np.uint8)
        join_off, j_agent, j_sigma = col("join_off", np.int32), col("join_agent", np.int32), \
            col("join_sigma", np.float64)
        delta_off, d_pool, base_caps = col("delta_off", np.int32), col("d_pool", np.int32), col("base_caps", np.int64)
        ch_off_all = col("ch_off", np.int32)
        ch_rows = col("ch_rows", np.int32).reshape(-1, 4)
        step_off, s_undo, s_retry, s_fail = col("step_off", np.int32), col("s_undo", np.uint8), \
            col("s_retry", np.int32), col("s_fail", np.uint8)
        nd_ = len(d_pool)
        cnt = np.diff(delta_off)
        turn = np.arange(nd_, dtype=np.int64) - np.repeat(delta_off[:-1].astype(np.int64), cnt) + 1
        digits = 1 + sum((turn >= 10 ** k).astype(np.int64) for k in range(1, 10)) if nd_ else np.zeros(0, np.int64)
        caps = ((base_caps + 2 * digits + np.where(turn > 1, 66, 4) + 8 + 63) & ~63).astype(np.int32)
    nd = len(caps)
    # Lane orders that balance the waves.  Render: records grouped by shape (turn 1 —
    # whole record hashed — first, then by change count and size), with their arena
    # space reserved in that same order so a wave's 64 records stay adjacent in the
    # arena.  Chain: sessions by descending serial work (later deltas).
    cnt_d = np.diff(delta_off).astype(np.int64)
    turn1 = np.zeros(nd, dtype=bool)
    if nd:
        turn1[delta_off[:-1][cnt_d > 0]] = True
    capl = caps.astype(np.int64)
    render_order = None
    # (the multi-key orders below are one stable argsort over a packed int64 key —
    # the same permutation as np.lexsort, at a fraction of its cost)
    cap_desc = (int(capl.max()) - capl) if nd else capl  # ≥ 0, < 2^40 (record reservations)
    t1_last = (~turn1).astype(np.int64) << 62
    if nd and _SP_ORDER & 2:
        nch = np.diff(np.asarray(ch_off_all, dtype=np.int64))
        render_order = np.argsort(t1_last | ((int(nch.max()) - nch) << 40) | cap_desc, kind="stable").astype(np.int32)
        rows_s, offs_s = st.reserve_deltas(caps[render_order])
        dr = np.empty(nd, dtype=np.int32)
        do = np.empty(nd, dtype=np.int64)
        dr[render_order] = np.frombuffer(rows_s, dtype=np.int32)
        do[render_order] = np.frombuffer(offs_s, dtype=np.int64)
        drows, doff = dr.tobytes(), do.tobytes()
    else:
        drows, doff = st.reserve_deltas(caps)
    dsess = np.repeat(np.arange(n, dtype=np.int32), np.diff(delta_off))

    has_saga = np.diff(step_off) > 0
    gslots = np.full(n, -1, dtype=np.int32)
    ng = int(has_saga.sum())
    if ng:
        gslots[has_saga] = st.alloc_many("G", ng)
    nsteps = int(step_off[-1])
    tslots = np.asarray(st.alloc_many("T", nsteps), dtype=np.int32) if nsteps else np.zeros(0, dtype=np.int32)

    def T(a, dtype=None):
        arr = np.array(a if dtype is None else np.asarray(a, dtype=dtype), copy=True, order="C")
        return torch.from_numpy(arr).to(dev)

    frag = None
    if nd and _SP_FRAGS and hasattr(C, "frag_pack"):
        frag = C.frag_pack(pool._pool, np.ascontiguousarray(d_pool, dtype=np.int32).tobytes(),
                           np.ascontiguousarray(ch_off_all, dtype=np.int32).tobytes(),
                           np.ascontiguousarray(ch_rows if len(ch_rows) else np.zeros((0, 4)),
                                                dtype=np.int32).tobytes())
    pb, po, pl = pool.device_view(dev)
    tens = {
        "slot": T(slots), "uuid": T(np.frombuffer(words, dtype=np.int32).reshape(n, 4)),
        "t0": T(np.full(n, t0, dtype=np.int64)), "creator": T(creator), "maxpart": T(maxpart), "minsig": T(minsig),
        "flags": T(flags), "join_off": T(join_off), "join_agent": T(j_agent), "join_sigma": T(j_sigma),
        "join_ring": torch.zeros(max(1, len(j_agent)), dtype=torch.uint8, device=dev),
        "join_code": torch.zeros(max(1, len(j_agent)), dtype=torch.uint8, device=dev),
        "delta_off": T(delta_off), "drow": T(np.frombuffer(drows, dtype=np.int32)), "dagent_pool": T(d_pool, np.int32),
        "dch_off": T(ch_off_all, np.int32),
        "changes": T(ch_rows if len(ch_rows) else np.zeros((1, 4), np.int32), np.int32),
        "doff": T(np.frombuffer(doff, dtype=np.int64)), "dcap": T(caps, np.int32), "dsess": T(dsess),
        "gslot": T(gslots), "step_off": T(step_off), "tslot": T(tslots if nsteps else np.zeros(1, np.int32)),
        "step_undo": T(s_undo if nsteps else np.zeros(1, np.uint8)),
        "step_retries": T(s_retry if nsteps else np.zeros(1, np.int32)),
        "step_fail": T(s_fail if nsteps else np.zeros(1, np.uint8)),
        "status": torch.zeros(n, dtype=torch.int32, device=dev),
        "pool_bytes": pb, "pool_off": po, "pool_len": pl,
    }
    # lane orders that balance the waves: sessions by descending chain work (SHA
    # blocks of their records), deltas by descending record size (stable sorts)
    # The render pass also compresses each record's parent-independent blocks (all
    # of a turn-1 record); the chain pass hashes the rest, ≈ the 4 blocks from the
    # parent hole on: chain work ∝ a session's later deltas.
    cs = np.concatenate([[0], np.cumsum((capl + 9 + 63) // 64 if _SP_PREFIX == "chain" else np.where(turn1, 0, 4))])
    work = cs[delta_off[1:]] - cs[delta_off[:-1]]
    if _SP_ORDER & 1:
        tens["chain_order"] = T(np.argsort(-work, kind="stable").astype(np.int32))
    if render_order is not None:
        tens["render_order"] = T(render_order)
    if _SP_PREFIX == "sorted" and nd:
        # prefix SHA lanes grouped by work: turn-1 records (hashed whole) first, then by
        # reserved size (∝ the blocks before the parent hole), so a wave's lanes finish together
        tens["prefix_order"] = T(np.argsort(t1_last | cap_desc, kind="stable").astype(np.int32))
    if frag is not None:
        tens["dfrag"] = T(np.frombuffer(frag["dfrag"], dtype=np.int32))
        tens["frag_bytes"] = T(np.frombuffer(frag["fbytes"], dtype=np.uint8))
        tens["frag_off"] = T(np.frombuffer(frag["foff"], dtype=np.int64))
        tens["frag_len"] = T(np.frombuffer(frag["flen"], dtype=np.int32))
    if _SP_PREFIX != "chain":
        tens["mid"] = torch.empty((max(1, nd), 8), dtype=torch.int32, device=dev)
        tens["mid_blocks"] = torch.zeros(max(1, nd), dtype=torch.int32, device=dev)
    args = {k: v.data_ptr() for k, v in tens.items()}
    args.update(prefix_in_render=_SP_PREFIX_IN_RENDER, render_first=_SP_OVERLAP,
                chain_roots=int(_SP_CHAIN_ROOTS),
                max_nch=int(np.diff(np.asarray(ch_off_all, dtype=np.int64)).max()) if nd else 0)
    args.update(n=n, nd=nd, gc_retention_us=int(hv.gc.policy.delta_retention_days) * 86_400 * 1_000_000)
    if shared:
        committed = list(range(n)) if (int(flags[0]) & 9) == 9 and delta_off[1] > 0 else []
    else:  # audit on, terminate requested, at least one delta (vectorized)
        committed = np.flatnonzero(((np.asarray(flags) & 9) == 9) & (np.diff(delta_off) > 0)).tolist()
    p = Prepared()
    p.store, p.specs, p.shared, p.n, p.nd, p.ids, p.slots, p.t0 = st, specs, shared, n, nd, ids, slots, t0
    p.tens, p.args, p.flags, p.committed, p.j_agent = tens, args, flags, committed, j_agent
    p.drows, p.doff, p.delta_off, p.gslots, p.step_off, p.tslots = drows, doff, delta_off, gslots, step_off, tslots
    p.g_live = tens["gslot"][tens["gslot"] >= 0] if ng else None
    p.t_live = tens["tslot"] if nsteps else None
    p.device_seconds = 0.0
    return p


def _k09_plan(p: "Prepared") -> Optional[tuple]:
    """(committed session indices, leaf delta rows, chain offsets, committed slots)
    on the device, built once per batch."""
    plan = p.__dict__.get("_k09")
    if plan is None and p.committed:
        st, tens, n, delta_off, committed = p.store, p.tens, p.n, p.delta_off, p.committed
        dev = st.device
        cix = torch.as_tensor(committed, dtype=torch.int64).to(dev)
        if p.shared:
            k = int(delta_off[1])
            leaves_idx = tens["drow"].view(n, k).index_select(0, cix).reshape(-1).to(torch.int64)
            offs = torch.arange(0, (len(committed) + 1) * k, k, dtype=torch.int32, device=dev)
        else:
            c = np.asarray(committed, dtype=np.int64)
            lo, hi = delta_off[c].astype(np.int64), delta_off[c + 1].astype(np.int64)
            lens = hi - lo
            if _SP_ORDER & 4:  # K09 lanes by chain length: a wave's trees have equal depth
                o = np.argsort(-lens, kind="stable")
                c, lo, hi, lens = c[o], lo[o], hi[o], lens[o]
                cix = torch.as_tensor(c, dtype=torch.int64).to(dev)
            # the committed chains' delta rows, concatenated (vectorized segment gather)
            seg = np.repeat(lo - np.concatenate([[0], np.cumsum(lens)[:-1]]), lens) + np.arange(int(lens.sum()))
            drow_np = np.frombuffer(p.drows, dtype=np.int32)
            leaves_idx = torch.as_tensor(drow_np[seg], dtype=torch.int64).to(dev)
            offs = torch.as_tensor(np.concatenate([[0], np.cumsum(lens)]), dtype=torch.int32).to(dev)
        plan = p.__dict__["_k09"] = (cix, leaves_idx, offs, tens["slot"].index_select(0, cix).to(torch.int64))
    return plan


def launch(p: "Prepared", sync: bool = True) -> "Prepared":
    """Run a prepared batch: rows / render / chain kernels, then K09 roots of the
    committed chains into ``s_root`` (stream-ordered; ``sync``: wait for them and
    let the store worker see the rows)."""
    import time

    st = p.store
    dev = st.device
    cuda = dev.type == "cuda"
    t_dev = time.perf_counter()
    if cuda:
        if sync:
            st.drain()
            st.flush()  # the worker's row writes (frees) are visible to the batch kernels
        st._c.run_pipeline(p.args, torch.cuda.current_stream(dev).cuda_stream)
    else:
        st._c.run_pipeline(p.args, 0)
    # K09: roots of the committed chains over the digests just written → s_root
    # (already there when the chain kernel folded them: chain_roots)
    plan = None if p.args.get("chain_roots") else _k09_plan(p)
    if plan is not None:
        from agent_hypervisor_amd.ops import audit as A

        _, leaves_idx, offs, sl = plan
        # leaves read in place from the resident digest table, roots written straight
        # into s_root (zeros for sessions that did not commit: terminate refused)
        A.merkle_roots(offs, st.tables["d_hash"].view(-1, 8), leaf_idx=leaves_idx,
                       root_out=st.tables["s_root"].view(-1, 8), root_row=sl, gate=st.tables["s_committed"])
    if cuda and sync:
        torch.cuda.synchronize(dev)
        st.acquire()  # the worker sees the batch's rows
    p.device_seconds = time.perf_counter() - t_dev
    return p


def finish(hv, p: "Prepared") -> PipelineRun:
    """Read back what the lazy views need and register the batch's sessions."""
    st, tens, n, nd, shared = p.store, p.tens, p.n, p.nd, p.shared
    specs, ids, slots, t0, committed = p.specs, p.ids, p.slots, p.t0, p.committed
    doff, delta_off, gslots, step_off, tslots = p.doff, p.delta_off, p.gslots, p.step_off, p.tslots
    drow_np = np.frombuffer(p.drows, dtype=np.int32)
    j_agent = p.j_agent
    # results the lazy views need, in one copy each
    status_np = tens["status"].cpu().numpy()
    dlen = tens["dcap"]  # replaced below by the rendered lengths
    hidx = (drow_np.astype(np.int64)[:, None] * 8 + np.arange(8, dtype=np.int64)[None, :]).reshape(-1)
    gath = st.gather({"d_len": drow_np, "d_hash": hidx}) \
        if nd else {"d_len": np.zeros(0, np.int32), "d_hash": np.zeros(0, np.int32)}
    dlen = gath["d_len"].astype(np.int64)
    dhash = gath["d_hash"].astype(np.uint32).reshape(-1, 8) if nd else np.zeros((0, 8), np.uint32)
    cidx = np.zeros(0, dtype=np.int64)
    flat = ""
    if committed:
        call = np.asarray(committed, dtype=np.int64)
        cs = slots[call].astype(np.int64)
        gg = st.gather({"s_root": (cs[:, None] * 8 + np.arange(8, dtype=np.int64)[None, :]).reshape(-1),
                        "s_committed": cs})
        keep = np.flatnonzero(gg["s_committed"])
        cidx = call[keep]
        rr = gg["s_root"].astype(np.uint32).reshape(-1, 8)[keep]
        flat = rr.byteswap().tobytes().hex()  # 8 BE words → 64 hex digits per root
    b = _Batch()
    b.store, b.specs, b.shared, b.ids, b.slots, b.t0 = st, specs, shared, ids, slots, t0
    b.doff, b.drows, b.dlen, b.dhash = np.frombuffer(doff, dtype=np.int64), drow_np, dlen, dhash
    b.delta_off, b.gslots, b.step_off, b.tslots = delta_off, gslots, step_off, tslots
    b.status, b.built, b.released, b.dead = status_np, np.zeros(n, dtype=bool), np.zeros(n, dtype=bool), []
    b._saga_ids = b._step_ids = None
    b.reserve_saga_ids()
    register_lazy(hv, b, status_np, cidx)
    run_ = PipelineRun(session_ids=ids, status=status_np,
                       join_rings=tens["join_ring"].cpu().numpy()[: len(j_agent)],
                       join_codes=tens["join_code"].cpu().numpy()[: len(j_agent)], device_seconds=p.device_seconds)
    run_._roots = (cidx, flat)
    return run_


# ------------------------------------------------------------------ lazy sessions


class _RowRef:
    """The identity of a lazy session's row (what batched reads need)."""

    __slots__ = ("slot", "session_id", "creator_did")

    def __init__(self, slot: int, session_id: str, creator_did: str) -> None:
        self.slot, self.session_id, self.creator_did = slot, session_id, creator_did


def register_lazy(hv, b: _Batch, status: np.ndarray, committed: np.ndarray) -> None:
    """Make the batch's sessions sessions of ``hv`` (no per-session objects);
    ``committed``: indices of the sessions whose roots the device committed."""
    ok = np.flatnonzero(status != 1)  # 1: row refused — nothing was written, the row stays with its owner
    ids = b.ids if len(ok) == len(b.ids) else [b.ids[i] for i in ok.tolist()]
    b.index = dict(zip(ids, ok.tolist()))
    b.views = {}
    b.committed = np.zeros(len(b.ids), dtype=bool)
    if len(committed):
        b.committed[committed] = True
        hv.commitment.register_batch(b)
    hv._sessions.add_batch(b, ids)


def materialize(b: _Batch, i: int) -> tuple:
    """Build the device views (session, delta engine, saga orchestrator) of batch
    session ``i`` (they take over its rows)."""
    from hypervisor import _device
    from hypervisor._clock import from_us
    from hypervisor.audit.delta import VFSChange
    from hypervisor.models import SessionConfig

    st = b.store
    sp = _spec(b, i)
    sid = b.ids[i]
    slot = int(b.slots[i])
    sso = _device.DeviceSession(st, sp.config or SessionConfig(), sp.creator_did, session_id=sid, slot=slot,
                                create=False)
    de = _device.DeviceDeltaEngine(st, slot, sid, sso)
    d0, d1 = int(b.delta_off[i]), int(b.delta_off[i + 1])
    prev = None
    specs_d = sp.deltas
    for k in range(d1 - d0):
        did, chs = specs_d[k]
        g = d0 + k
        ts = from_us(int(b.t0) + 1 + k)
        changes = [VFSChange(path=c[0], operation=c[1], content_hash=c[2],
                             previous_hash=c[3] if len(c) > 3 else None) for c in chs]
        d = _device.DeviceDelta(de, f"delta:{k + 1}", k + 1, sid, did, ts, changes, prev)
        h = "".join(f"{int(w):08x}" for w in b.dhash[g])
        d.__dict__.update(_didx=int(b.drows[g]), _poff=int(b.doff[g]), _plen=int(b.dlen[g]), _seq=-1, _dev_hash=h)
        de._deltas.append(d)
        de._rows.append(int(b.drows[g]))
        prev = d
    de._turn_counter = d1 - d0
    orch = _device.DeviceSagaOrchestrator(st, sso)
    g = int(b.gslots[i])
    if g >= 0:
        gids, tids = b.saga_ids()
        saga = _device.DeviceSaga(st, g, gids[i], sid)
        for k in range(int(b.step_off[i]), int(b.step_off[i + 1])):
            a = sp.steps[k - int(b.step_off[i])]
            step = _device.DeviceSagaStep(st, int(b.tslots[k]), step_id=tids[k], action_id=a[0],
                                          agent_did=a[1], execute_api=a[2], undo_api=a[3], timeout_seconds=300,
                                          max_retries=int(a[4]))
            saga.steps.append(step)
        orch._sagas[saga.saga_id] = saga
    return sso, de, orch


