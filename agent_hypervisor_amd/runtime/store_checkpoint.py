"""Columnar checkpoint of a device-backed hypervisor (``Hypervisor(device=...)``).

The per-session JSON format (:mod:`agent_hypervisor_amd.runtime.checkpoint`)
reads every session through its views — several store round trips and a Python
record per session.  This one dumps the *store* instead: the live rows of every
table, gathered column by column (one tensor gather per column, no store
command per session), the payload-arena records — which are exactly the
canonical-JSON bytes each digest was computed over — and the few Python-side
fields the rows do not hold (string ids, saga/step descriptors, VFS contents).

Files (listed in the manifest with their SHA-256):

``store.safetensors``
    ``S.<col>`` / ``P.<col>`` / ``D.<col>`` / ``G.<col>`` / ``T.<col>``: the
    columns of the saved sessions' rows, their participant rows (ragged), their
    delta chains in chain order, sagas and steps; ``off.*`` the ragged offsets
    (deltas / participants / sagas per session, steps per saga); ``str.*``
    dictionary-encoded string columns (session / saga / step ids, DIDs, APIs).
    Row *indices* are not saved: restore allocates rows in the target store and
    rewrites every row reference (``s_dlast``, ``d_sess``, ``d_prev``, ``d_off``,
    ``t_saga``, agent ids).
``arena.bin``
    the chains' records, concatenated in ``D`` order (``D.d_len`` each).  Its
    manifest entry is ``"k10"``: every byte belongs to one record and restore
    re-hashes every record against its (manifest-protected) digest, so the
    chain re-verification *is* the integrity check of this file.
``store.json``
    counts, vouch records in creation order, commitments held outside session
    rows, per-session VFS / reversibility extras.

Restore (:func:`load_store`): rows are allocated in bulk, the columns written
with one ``index_copy_`` per column (:meth:`GovernanceStore.write_columns`), the
records with one native copy, every chain re-verified — record digests, parent
quotes and committed Merkle roots (K10 + K09) — on host threads over the same
bytes, and the sessions registered *lazily* (:class:`RestoredBatch`): their
views are built from the rows on first use, like the batched pipeline's.

Reference: the reference keeps all state in memory and has no checkpoint
(``src/hypervisor/saga/state_machine.py:133-152`` is its only persistence hook);
SURVEY §5.4.
"""

from __future__ import annotations

import json
import math
import os
from datetime import datetime
from typing import Any, Optional

import numpy as np
import torch

from agent_hypervisor_amd._native import C

LAYOUT = "columnar"
FILES = ("store.safetensors", "arena.bin", "store.json")

# columns restored verbatim (row references are rewritten separately)
S_COLS = ("s_state", "s_mode", "s_audit", "s_maxpart", "s_minsig", "s_creator", "s_created", "s_terminated",
          "s_pcount", "s_pactive", "s_dcount", "s_committed", "s_commit_n", "s_released", "s_retained")
S_WIDE = {"s_uuid": 4, "s_head": 8, "s_root": 8}
P_COLS = ("p_agent", "p_ring", "p_active", "p_sraw", "p_seff", "p_joined")
D_COLS = ("d_turn", "d_ts", "d_len", "d_hole")
G_COLS = ("g_state", "g_created", "g_completed", "g_nsteps")
T_COLS = ("t_state", "t_undo", "t_started", "t_completed", "t_retry", "t_maxretry")
_MODES = ("eventual", "strong")


from agent_hypervisor_amd.runtime.checkpoint import CheckpointError  # noqa: E402


# ---------------------------------------------------------------- strings


class _Strs:
    """A dictionary-encoded string column being collected: ``codes`` index a
    table of distinct-or-not strings (``None`` allowed)."""

    def __init__(self) -> None:
        self.table: list = []
        self.codes: list = []

    def one(self, s: Optional[str]) -> None:
        self.codes.append(np.asarray([len(self.table)], dtype=np.int64))
        self.table.append(s)

    def many(self, strs: list) -> None:
        b = len(self.table)
        self.table.extend(strs)
        self.codes.append(np.arange(b, b + len(strs), dtype=np.int64))

    def coded(self, codes: np.ndarray, table: list) -> None:
        b = len(self.table)
        self.table.extend(table)
        self.codes.append(np.asarray(codes, dtype=np.int64) + b)

    def const(self, s: Optional[str], n: int) -> None:
        if n:
            self.coded(np.zeros(n, dtype=np.int64), [s])

    def tensors(self, name: str) -> dict:
        codes = np.concatenate(self.codes) if self.codes else np.zeros(0, np.int64)
        tab = self.table
        if None in tab:
            null = np.fromiter((s is None for s in tab), dtype=np.uint8, count=len(tab))
            lens = np.fromiter((0 if s is None else len(s) for s in tab), dtype=np.int64, count=len(tab))
            blob = "".join(s for s in tab if s is not None)
        else:  # the common case (ids): no null entries
            null = np.zeros(len(tab), dtype=np.uint8)
            lens = np.fromiter(map(len, tab), dtype=np.int64, count=len(tab))
            blob = "".join(tab)
        off = np.zeros(len(tab) + 1, dtype=np.int64)
        np.cumsum(lens, out=off[1:])
        blob = blob.encode("utf-8", "surrogatepass")
        return {f"str.{name}.codes": torch.from_numpy(codes), f"str.{name}.off": torch.from_numpy(off),
                f"str.{name}.null": torch.from_numpy(null),
                f"str.{name}.blob": torch.frombuffer(bytearray(blob), dtype=torch.uint8) if blob
                else torch.zeros(0, dtype=torch.uint8)}


class _Col:
    """A restored string column: ``col[i]`` decodes entry ``i`` on demand."""

    __slots__ = ("codes", "text", "off", "null", "ctr", "seed", "_mint", "_minted")

    def __init__(self, t: dict, name: str, mint: Optional[str] = None) -> None:
        self.codes = t[f"str.{name}.codes"].numpy()
        blob = t[f"str.{name}.blob"].numpy().tobytes()
        self.text = blob.decode("utf-8", "surrogatepass")
        self.off = t[f"str.{name}.off"].numpy()
        self.null = t[f"str.{name}.null"].numpy()
        c = t.get(f"ctr.{name}")
        self.ctr = c.numpy() if c is not None else np.full(len(self.codes), -1, dtype=np.int64)
        sd = t.get(f"seed.{name}")
        self.seed = sd.numpy() if sd is not None else np.zeros(len(self.codes), dtype=np.int64)
        self._mint = mint  # id prefix: entries held as (seed, counter) are formatted on demand
        self._minted: dict = {}

    def table(self) -> list:
        off = self.off.tolist()
        nul = self.null
        return [None if nul[k] else self.text[off[k]:off[k + 1]] for k in range(len(nul))]

    def __len__(self) -> int:
        return len(self.codes)

    def at(self, code: int) -> Optional[str]:
        if self.null[code]:
            return None
        return self.text[int(self.off[code]):int(self.off[code + 1])]

    def __getitem__(self, i: int) -> Optional[str]:
        k = int(self.ctr[i])
        if k >= 0:
            return C.uuid_from_counter(int(np.int64(self.seed[i]).view(np.uint64)), k, self._mint or "")
        c = int(self.codes[i])
        if self.null[c] and self._mint is not None:  # no id was ever formatted: a fresh one, kept
            s = self._minted.get(i)
            if s is None:
                s = self._minted[i] = C.uuid4(self._mint)
            return s
        return self.at(c)

    def all(self) -> list:
        """Every entry (the table decoded once, then indexed)."""
        off = self.off.tolist()
        txt = self.text
        nul = self.null
        if nul.any():
            tab = [None if nul[k] else txt[off[k]:off[k + 1]] for k in range(len(nul))]
        else:
            tab = [txt[a:b] for a, b in zip(off, off[1:])]
        c = self.codes
        if len(c) == len(tab) and (len(c) == 0 or (c[0] == 0 and (np.diff(c) == 1).all())):
            return tab  # one entry per code, in order (unique ids)
        return [tab[k] for k in c.tolist()]

    def take(self, idx: np.ndarray) -> "_Col":
        c = object.__new__(_Col)
        c.codes, c.text, c.off, c.null, c._mint, c._minted = self.codes[idx], self.text, self.off, self.null, \
            self._mint, {}
        c.ctr, c.seed = self.ctr[idx], self.seed[idx]
        return c


# ---------------------------------------------------------------- collection


def _us(t: Optional[datetime]) -> Optional[int]:
    from hypervisor._clock import to_us

    return to_us(t) if t is not None else None


def _jsonable(x: Any) -> Any:
    try:
        json.dumps(x)
        return x
    except (TypeError, ValueError):
        return {"__repr__": repr(x)}


class _Collect:
    """Per-session host metadata of the saved sessions, in table order."""

    def __init__(self) -> None:
        self.ids: list = []
        self.slots: list = []
        self.cfg_mode: list = []
        self.cfg_maxdur: list = []
        self.cfg_chain: list = []
        self.dskip: list = []
        self.g_sess: list = []
        self.g_row: list = []
        self.g_id = _Strs()
        self.g_ctr: list = []  # (seed, counter) of ids formatted on demand; counter -1: a string id
        self.g_seed: list = []
        self.g_err = _Strs()
        self.t_saga: list = []
        self.t_row: list = []
        self.t_timeout: list = []
        self.t_ctr: list = []
        self.t_seed: list = []
        self.t_str = {k: _Strs() for k in ("step_id", "action_id", "agent_did", "execute_api", "undo_api", "error",
                                           "execute_result", "compensation_result")}
        self.extras: dict = {}
        self.drows: list = []  # each session's delta rows in chain order (host-known: no device walk)
        self.dcnt: list = []
        self.n = 0
        self.ng = 0

    # one materialised session (ordinary, or a batch session whose views exist)
    def view(self, m) -> None:
        from hypervisor.models import ConsistencyMode

        sso = m.sso
        cfg = sso.config
        i = self.n
        self.ids.append(sso.session_id)
        self.slots.append(np.asarray([sso.slot], dtype=np.int64))
        self.cfg_mode.append(np.asarray([int(ConsistencyMode(cfg.consistency_mode) is ConsistencyMode.STRONG)],
                                        dtype=np.uint8))
        md = cfg.max_duration_seconds
        self.cfg_maxdur.append(np.asarray([math.nan if md is None else float(md)]))
        self.cfg_chain.append(np.asarray([int(bool(cfg.enable_blockchain_commitment))], dtype=np.uint8))
        de = m.delta_engine
        rows = list(getattr(de, "_rows", ()))
        self.dskip.append(np.asarray([len(rows) - len(de._deltas)], dtype=np.int32))
        self.drows.append(np.asarray(rows, dtype=np.int64))
        self.dcnt.append(np.asarray([len(rows)], dtype=np.int64))
        for g in m.saga._sagas.values():
            self.g_sess.append(np.asarray([i], dtype=np.int64))
            self.g_row.append(np.asarray([g.slot], dtype=np.int64))
            self.g_id.one(g.saga_id)
            self._ctr(self.g_ctr, self.g_seed, 1)
            self.g_err.one(g.error)
            for s in g.steps:
                self._ctr(self.t_ctr, self.t_seed, 1)
                self.t_saga.append(np.asarray([self.ng], dtype=np.int64))
                self.t_row.append(np.asarray([s.slot], dtype=np.int64))
                self.t_timeout.append(np.asarray([float(s.timeout_seconds)]))
                ts = self.t_str
                ts["step_id"].one(s.step_id)
                ts["action_id"].one(s.action_id)
                ts["agent_did"].one(s.agent_did)
                ts["execute_api"].one(s.execute_api)
                ts["undo_api"].one(s.undo_api)
                ts["error"].one(s.error)
                ts["execute_result"].one(json.dumps(_jsonable(s.execute_result)))
                ts["compensation_result"].one(json.dumps(_jsonable(s.compensation_result)))
            self.ng += 1
        ex = _extras(m)
        if ex:
            self.extras[i] = ex
        self.n += 1

    # unbuilt sessions of a batched pipeline (store_pipeline._Batch), vectorized
    def batch(self, b, idx: np.ndarray) -> None:
        from agent_hypervisor_amd.models import store_pipeline as SP
        from agent_hypervisor_amd.models.store_template import _TemplateSpecs
        from hypervisor.models import ConsistencyMode, SessionConfig

        k = len(idx)
        if not k:
            return
        base = self.n
        self.n += k
        ids = b.ids
        self.ids.extend(ids[i] for i in idx.tolist())
        self.slots.append(b.slots[idx].astype(np.int64))
        uniform = b.shared or isinstance(b.specs, _TemplateSpecs)
        if uniform:
            cfgs = [(b.specs.config if b.shared else b.specs.tp.config) or SessionConfig()] * k
        else:
            cfgs = [SP._spec(b, i).config or SessionConfig() for i in idx.tolist()]
        c0 = cfgs[0] if uniform else None
        if uniform:
            mode = int(ConsistencyMode(c0.consistency_mode) is ConsistencyMode.STRONG)
            md = c0.max_duration_seconds
            self.cfg_mode.append(np.full(k, mode, dtype=np.uint8))
            self.cfg_maxdur.append(np.full(k, math.nan if md is None else float(md)))
            self.cfg_chain.append(np.full(k, int(bool(c0.enable_blockchain_commitment)), dtype=np.uint8))
        else:
            self.cfg_mode.append(np.asarray([int(ConsistencyMode(c.consistency_mode) is ConsistencyMode.STRONG)
                                             for c in cfgs], dtype=np.uint8))
            self.cfg_maxdur.append(np.asarray([math.nan if c.max_duration_seconds is None
                                               else float(c.max_duration_seconds) for c in cfgs]))
            self.cfg_chain.append(np.asarray([int(bool(c.enable_blockchain_commitment)) for c in cfgs],
                                             dtype=np.uint8))
        self.dskip.append(np.zeros(k, dtype=np.int32))
        self._batch_drows(b, idx)
        # sagas: at most one per batch session, its steps from the spec
        g = b.gslots[idx]
        has = np.flatnonzero(g >= 0)
        if not len(has):
            return
        hi = idx[has]
        ng = len(has)
        self.g_sess.append(base + has.astype(np.int64))
        self.g_row.append(g[has].astype(np.int64))
        counters = b._saga_ids is None and getattr(b, "id_seed", None) is not None
        if counters:  # not formatted yet: save the id generator's counters (same ids either side)
            gids = tids = None
            self.g_id.const(None, ng)
            self._ctr(self.g_ctr, self.g_seed, ng, b.id_seed, b.gid_base + hi.astype(np.int64))
        else:
            gids, tids = b.saga_ids()
            self.g_id.many([gids[i] for i in hi.tolist()])
            self._ctr(self.g_ctr, self.g_seed, ng)
        self.g_err.const(None, ng)
        s0, s1 = b.step_off[hi].astype(np.int64), b.step_off[hi + 1].astype(np.int64)
        cnt = s1 - s0
        nt = int(cnt.sum())
        tix = np.repeat(s0 - np.concatenate([[0], np.cumsum(cnt)[:-1]]), cnt) + np.arange(nt)  # step rows
        self.t_saga.append(np.repeat(self.ng + np.arange(ng, dtype=np.int64), cnt))
        self.t_row.append(b.tslots[tix].astype(np.int64))
        self.t_timeout.append(np.full(nt, 300.0))
        ts = self.t_str
        if tids is not None:
            ts["step_id"].many([tids[j] for j in tix.tolist()])
            self._ctr(self.t_ctr, self.t_seed, nt)
        else:
            ts["step_id"].const(None, nt)
            self._ctr(self.t_ctr, self.t_seed, nt, b.id_seed, b.tid_base + tix.astype(np.int64))
        for key in ("error",):
            ts[key].const(None, nt)
        ts["execute_result"].const("null", nt)
        ts["compensation_result"].const("null", nt)
        if b.shared or isinstance(b.specs, _TemplateSpecs):
            if b.shared:
                steps = list(b.specs.steps)
                per = np.tile(np.arange(len(steps)), ng) if steps else np.zeros(0, np.int64)
                ts["action_id"].coded(per, [x[0] for x in steps])
                ts["agent_did"].coded(per, [x[1] for x in steps])
                ts["execute_api"].coded(per, [x[2] for x in steps])
                ts["undo_api"].coded(per, [x[3] for x in steps])
            else:  # template: one step ("action", the session's agent, "/api/action", no undo)
                tp = b.specs.tp
                ts["action_id"].const("action", nt)
                ts["agent_did"].coded(np.repeat(b.specs.agent_idx[hi], cnt), list(tp.agents.dids))
                ts["execute_api"].const("/api/action", nt)
                ts["undo_api"].const(None, nt)
        else:
            for i, c in zip(hi.tolist(), cnt.tolist()):
                steps = SP._spec(b, i).steps
                for x in steps[:c]:
                    ts["action_id"].one(x[0])
                    ts["agent_did"].one(x[1])
                    ts["execute_api"].one(x[2])
                    ts["undo_api"].one(x[3])
        self.ng += ng

    # unbuilt sessions of a restored batch
    def restored(self, b: "RestoredBatch", idx: np.ndarray) -> None:
        k = len(idx)
        if not k:
            return
        base = self.n
        self.n += k
        ids = b.ids
        self.ids.extend(ids[i] for i in idx.tolist())
        self.slots.append(b.slots[idx].astype(np.int64))
        self.cfg_mode.append(b.cfg_mode[idx])
        self.cfg_maxdur.append(b.cfg_maxdur[idx])
        self.cfg_chain.append(b.cfg_chain[idx])
        self.dskip.append(b.dskip[idx])
        self._batch_drows(b, idx)
        g0, g1 = b.goff[idx], b.goff[idx + 1]
        gcnt = g1 - g0
        ng = int(gcnt.sum())
        if b.extras:  # position of each batch index in `idx` (any order)
            for k, i in enumerate(idx.tolist()):
                ex = b.extras.get(i)
                if ex is not None:
                    self.extras[base + k] = ex
        if not ng:
            return
        gix = np.repeat(g0 - np.concatenate([[0], np.cumsum(gcnt)[:-1]]), gcnt) + np.arange(ng)
        self.g_sess.append(base + np.repeat(np.arange(k, dtype=np.int64), gcnt))
        self.g_row.append(b.gslots[gix].astype(np.int64))
        self.g_id.coded(b.gid.codes[gix], b.gid.table())
        self.g_ctr.append(b.gid.ctr[gix])
        self.g_seed.append(b.gid.seed[gix])
        self.g_err.many([b.gerr[j] for j in gix.tolist()])
        t0, t1 = b.toff[gix], b.toff[gix + 1]
        tcnt = t1 - t0
        nt = int(tcnt.sum())
        tix = np.repeat(t0 - np.concatenate([[0], np.cumsum(tcnt)[:-1]]), tcnt) + np.arange(nt)
        self.t_saga.append(np.repeat(self.ng + np.arange(ng, dtype=np.int64), tcnt))
        self.t_row.append(b.tslots[tix].astype(np.int64))
        self.t_timeout.append(b.t_timeout[tix])
        for key, col in b.tcols.items():
            self.t_str[key].coded(col.codes[tix], col.table())
        sid = b.tcols["step_id"]
        self.t_ctr.append(sid.ctr[tix])
        self.t_seed.append(sid.seed[tix])
        self.ng += ng


def _batch_drows(self, b, idx: np.ndarray) -> None:
    """Delta rows of batch sessions ``idx`` (chain order), from the batch's arrays."""
    off = np.asarray(b.delta_off, dtype=np.int64)
    cnt = off[idx + 1] - off[idx]
    self.dcnt.append(cnt)
    self.drows.append(np.asarray(b.drows, dtype=np.int64)[_ragged(off[idx], cnt)] if int(cnt.sum())
                      else np.zeros(0, np.int64))


_Collect._batch_drows = _batch_drows


def _ctr_append(ctr: list, seed: list, n: int, s: Optional[int] = None, c: Optional[np.ndarray] = None) -> None:
    if not n:
        return
    if s is None:
        ctr.append(np.full(n, -1, dtype=np.int64))
        seed.append(np.zeros(n, dtype=np.int64))
    else:
        ctr.append(np.asarray(c, dtype=np.int64))
        seed.append(np.full(n, np.int64(np.uint64(s).view(np.int64)), dtype=np.int64))


_Collect._ctr = staticmethod(_ctr_append)


def _extras(m) -> Optional[dict]:
    """VFS contents / edit log and reversibility entries (host-side session state)."""
    from hypervisor.core import LazyManagedSession

    if isinstance(m, LazyManagedSession):
        return None
    sso = m.sso
    out = {}
    vfs = sso.vfs
    if vfs._files or vfs._permissions or vfs.edit_log:
        out["vfs"] = {
            "files": dict(vfs._files),
            "permissions": {k: sorted(v) for k, v in vfs._permissions.items()},
            "edits": [{"path": e.path, "operation": e.operation, "agent_did": e.agent_did,
                       "timestamp": e.timestamp.isoformat() if e.timestamp else None,
                       "content_hash": e.content_hash, "previous_hash": e.previous_hash} for e in vfs.edit_log],
        }
    ents = m.reversibility.entries
    if ents:
        out["reversibility"] = [
            {"action_id": e.action_id, "execute_api": e.execute_api, "undo_api": e.undo_api,
             "reversibility": e.reversibility.value, "undo_window_seconds": e.undo_window_seconds,
             "compensation_method": e.compensation_method, "undo_api_healthy": e.undo_api_healthy}
            for e in ents]
    return out or None


def _ragged(off_lo: np.ndarray, cnt: np.ndarray) -> np.ndarray:
    """Concatenated ranges [off_lo[i], off_lo[i] + cnt[i])."""
    n = int(cnt.sum())
    if not n:
        return np.zeros(0, dtype=np.int64)
    starts = np.concatenate([[0], np.cumsum(cnt)[:-1]])
    return np.repeat(off_lo.astype(np.int64) - starts, cnt) + np.arange(n, dtype=np.int64)


def _take(st, name: str, rows: np.ndarray, width: int = 1, device: bool = False) -> torch.Tensor:
    """Rows of a store column (``width`` words per row), gathered on the device;
    copied to the host unless ``device``."""
    t = st.tables[name]
    ix = torch.from_numpy(np.ascontiguousarray(rows, dtype=np.int64)).to(t.device)
    out = t.view(-1, width).index_select(0, ix) if width > 1 else t.index_select(0, ix)
    return out.contiguous() if device else out.cpu().contiguous()


# host-side copies of these columns travel with the host part even when the
# columns themselves stay on the device (the receiver's allocators and lazy views
# need them; a few bytes per row)
HOST_COLS = ("S.s_pcount", "S.s_dcount", "S.s_maxpart", "S.s_minsig", "S.s_audit", "S.s_committed",
             "S.s_commit_n", "D.d_len")


def _selected(hv, only: Optional[set]) -> _Collect:
    """The sessions to save (all of ``hv``'s, or the ids in ``only``), collected in
    creation order: built views through their objects, unbuilt batch sessions
    vectorized."""
    from agent_hypervisor_amd.models.store_pipeline import _Batch

    col = _Collect()
    for kind, seg in hv._sessions.segments():
        if kind == "own":
            for m in seg:
                if only is None or m.sso.session_id in only:
                    col.view(m)
            continue
        order = np.fromiter(seg.index.values(), dtype=np.int64, count=len(seg.index))
        if only is not None:
            ids = seg.ids
            order = order[np.fromiter((ids[i] in only for i in order.tolist()), dtype=bool, count=len(order))]
        built = np.fromiter((i in seg.views for i in order.tolist()), dtype=bool, count=len(order))
        # runs of unbuilt sessions vectorized, built ones through their views (creation order kept)
        edges = np.flatnonzero(np.diff(built.astype(np.int8))) + 1
        for run in np.split(np.arange(len(order)), edges):
            if not len(run):
                continue
            ix = order[run]
            if built[run[0]]:
                for i in ix.tolist():
                    col.view(seg.views[i])
            elif isinstance(seg, RestoredBatch):
                col.restored(seg, ix)
            elif isinstance(seg, _Batch):
                col.batch(seg, ix)
            else:
                raise CheckpointError(f"unknown session segment {type(seg).__name__}")
    return col


def collect(hv, only: Optional[set] = None, device: bool = False) -> tuple:
    """The columnar image of ``hv``'s sessions (``only``: just these ids, with their
    vouches, commitments and extras): ``(cols, host, arena, meta)``.

    * ``cols`` — every table column of the sessions' rows (``S.*`` sessions,
      ``P.*`` participants, ``D.*`` delta chains in chain order, ``G.*`` sagas,
      ``T.*`` steps), gathered on the device and left there with ``device`` (the
      migration path: nothing crosses to the host), copied to the host otherwise;
    * ``host`` — host tensors: ragged offsets, configs, dictionary-encoded string
      columns (ids, DIDs, descriptors) and the :data:`HOST_COLS` copies;
    * ``arena`` — the chains' records concatenated in ``D`` order: a device uint8
      tensor with ``device`` (one record-move kernel), else bytes;
    * ``meta`` — counts, vouch records, host-held commitments, VFS/reversibility extras.
    """
    st = hv._store
    st.verify_deferred(block=True)
    col = _selected(hv, only)
    n = len(col.ids)
    assert col.n == n
    cat = lambda xs, dt: np.concatenate(xs).astype(dt) if xs else np.zeros(0, dt)  # noqa: E731
    slots = cat(col.slots, np.int64)
    st.drain()
    if st.device.type == "cuda":
        st.flush()
    take = lambda name, rows, w=1: _take(st, name, rows, w, device)  # noqa: E731
    T: dict = {}
    # -- sessions ------------------------------------------------------------------
    for name in S_COLS:
        T[f"S.{name}"] = take(name, slots)
    for name, w in S_WIDE.items():
        T[f"S.{name}"] = take(name, slots, w)
    S_cap = st.caps["S"]
    pcnt = T["S.s_pcount"].cpu().numpy().astype(np.int64)
    kpos = np.arange(int(pcnt.sum()), dtype=np.int64) - np.repeat(np.concatenate([[0], np.cumsum(pcnt)[:-1]]), pcnt)
    prow = kpos * S_cap + np.repeat(slots, pcnt)  # participant-major columns (store.h prow)
    for name in P_COLS:
        T[f"P.{name}"] = take(name, prow)
    # -- delta chains, in chain order (the rows each session's views / batch hold) ----
    dcnt = cat(col.dcnt, np.int64)
    drow = cat(col.drows, np.int64)
    dev_cnt = T["S.s_dcount"].to(torch.int64).cpu().numpy()
    if len(dcnt) != n or not np.array_equal(dcnt, dev_cnt):
        raise CheckpointError("delta chains differ from their sessions' delta counts (store corrupt)")
    doff = np.zeros(n + 1, dtype=np.int64)
    np.cumsum(dcnt, out=doff[1:])
    nd = int(doff[-1])
    for name in D_COLS:
        T[f"D.{name}"] = take(name, drow)
    T["D.d_hash"] = take("d_hash", drow, 8)
    dlen = T["D.d_len"].to(torch.int64).cpu().numpy()
    aoff_src = take("d_off", drow).to(torch.int64)
    if device:
        from agent_hypervisor_amd.ops.store_views import move_records

        arena = move_records(st, aoff_src, torch.from_numpy(dlen).to(st.device), None)
    else:
        arena = st._c.payload_gather(aoff_src.numpy(), dlen) if nd else b""
    # -- sagas / steps ---------------------------------------------------------------
    g_row, t_row = cat(col.g_row, np.int64), cat(col.t_row, np.int64)
    g_sess, t_saga = cat(col.g_sess, np.int64), cat(col.t_saga, np.int64)
    for name in G_COLS:
        T[f"G.{name}"] = take(name, g_row)
    for name in T_COLS:
        T[f"T.{name}"] = take(name, t_row)
    goff = np.zeros(n + 1, dtype=np.int64)
    np.cumsum(np.bincount(g_sess, minlength=n), out=goff[1:])
    toff = np.zeros(len(g_row) + 1, dtype=np.int64)
    np.cumsum(np.bincount(t_saga, minlength=len(g_row)), out=toff[1:])
    if (np.diff(g_sess) < 0).any() or (np.diff(t_saga) < 0).any():
        raise CheckpointError("saga rows collected out of session order")
    H: dict = {}
    H["off.delta"] = torch.from_numpy(doff)
    H["off.part"] = torch.from_numpy(np.concatenate([[0], np.cumsum(pcnt)]).astype(np.int64))
    H["off.saga"] = torch.from_numpy(goff)
    H["off.step"] = torch.from_numpy(toff)
    H["sess.cfg_mode"] = torch.from_numpy(cat(col.cfg_mode, np.uint8))
    H["sess.cfg_maxdur"] = torch.from_numpy(cat(col.cfg_maxdur, np.float64))
    H["sess.cfg_chain"] = torch.from_numpy(cat(col.cfg_chain, np.uint8))
    H["sess.dskip"] = torch.from_numpy(cat(col.dskip, np.int32))
    H["step.timeout"] = torch.from_numpy(cat(col.t_timeout, np.float64))
    ids = _Strs()
    ids.many(col.ids)
    H.update(ids.tensors("session_id"))
    H.update(col.g_id.tensors("saga_id"))
    H["ctr.saga_id"] = torch.from_numpy(cat(col.g_ctr, np.int64))
    H["seed.saga_id"] = torch.from_numpy(cat(col.g_seed, np.int64))
    H["ctr.step.step_id"] = torch.from_numpy(cat(col.t_ctr, np.int64))
    H["seed.step.step_id"] = torch.from_numpy(cat(col.t_seed, np.int64))
    H.update(col.g_err.tensors("saga_error"))
    for k, s_ in col.t_str.items():
        H.update(s_.tensors(f"step.{k}"))
    # -- agents referenced by the rows: dictionary codes (re-interned by the reader) ----
    ag = torch.cat([T["S.s_creator"].to(torch.int64), T["P.p_agent"].to(torch.int64)])
    if ag.numel():
        uniq, inv = torch.unique(ag, return_inverse=True)
    else:
        uniq, inv = ag, ag
    T["S.s_creator"] = inv[:n].to(torch.int32).contiguous()
    T["P.p_agent"] = inv[n:].to(torch.int32).contiguous()
    agents = _Strs()
    agents.many([st.did(int(a)) for a in uniq.cpu().tolist()])
    H.update(agents.tensors("agents"))
    for k in HOST_COLS:
        H["host." + k] = T[k].cpu()
    meta = {
        "layout": LAYOUT, "sessions": n, "deltas": nd, "sagas": len(g_row), "steps": len(t_row),
        "participant_rows": st.caps["P"], "arena_bytes": int(dlen.sum()) if nd else 0,
        "batched_sessions": int(getattr(hv, "batched_sessions", 0)),
        "vouches": _vouches(hv, only), "commitments": _host_commitments(hv, only),
        "extras": {str(k): v for k, v in col.extras.items()},
    }
    return T, H, arena, meta


def save_store(hv, d: str) -> dict:
    """Write the columnar files of ``hv`` (device-backed) into directory ``d``;
    returns the manifest extras (``{"layout", "sessions"}``) and the file digests
    the caller lists."""
    from safetensors.torch import save_file

    T, H, arena, meta = collect(hv)
    T.update({k: v for k, v in H.items() if not k.startswith("host.")})
    save_file(T, os.path.join(d, "store.safetensors"), metadata={"format": "ahv-checkpoint", "layout": LAYOUT})
    with open(os.path.join(d, "arena.bin"), "wb") as f:
        f.write(arena)
    with open(os.path.join(d, "store.json"), "w") as f:
        json.dump(meta, f)
    return {"layout": LAYOUT, "sessions": meta["sessions"]}


def _vouches(hv, only: Optional[set] = None) -> list:
    """Vouch records in creation order (of the sessions ``only``, when given); bond
    state from the edge rows (one gather)."""
    ve = hv.vouching
    recs = list(getattr(ve, "_order", ()))
    if only is not None:
        recs = [r for r in recs if r.session_id in only]
    st = hv._store
    live = [r.edge for r in recs if getattr(r, "edge", -1) >= 0]
    g = st.gather({"e_active": live, "e_released": live}) if live else {}
    out, k = [], 0
    for r in recs:
        if getattr(r, "edge", -1) >= 0:
            act, rel = int(g["e_active"][k]), int(g["e_released"][k])
            k += 1
        else:
            f = r._frozen
            act, rel = int(f[1]), int(np.int64(np.uint64(f[2])))
        out.append({"vouch_id": r.vouch_id, "voucher_did": r.voucher_did, "vouchee_did": r.vouchee_did,
                    "session_id": r.session_id, "pct": r.bonded_sigma_pct, "bonded": r.bonded_amount,
                    "created_us": _us(r.created_at), "expiry_us": _us(r.expiry), "active": act,
                    "released_us": rel, "linked": getattr(r, "edge", -1) >= 0})
    return out


def _host_commitments(hv, only: Optional[set] = None) -> list:
    from agent_hypervisor_amd.runtime.checkpoint import _iso

    out = []
    for c in getattr(hv.commitment, "_commitments", {}).values():
        if only is not None and c.session_id not in only:
            continue
        out.append({"session_id": c.session_id, "merkle_root": c.merkle_root, "participant_dids": c.participant_dids,
                    "delta_count": c.delta_count, "committed_at": _iso(c.committed_at),
                    "blockchain_tx_id": c.blockchain_tx_id, "committed_to": c.committed_to})
    return out


# ---------------------------------------------------------------- restore


def read_tables(d: str) -> tuple:
    from safetensors.torch import load_file

    t = load_file(os.path.join(d, "store.safetensors"))
    with open(os.path.join(d, "store.json")) as f:
        meta = json.load(f)
    return t, meta


def session_keys(d: str) -> list:
    t, meta = read_tables(d)
    keys = _Col(t, "session_id").all()
    seen = set(keys)
    for v in meta["vouches"]:
        if v["session_id"] not in seen:
            seen.add(v["session_id"])
            keys.append(v["session_id"])
    return keys


def load_store(hv, d: str, verify: bool = True, only=None):
    """Restore the columnar checkpoint in ``d`` into the device-backed ``hv``
    (``only``: just these session ids, with their vouches and commitments).  The
    arena file's integrity check is the host K10/K09 re-verification (always)."""
    t, meta = read_tables(d)
    with open(os.path.join(d, "arena.bin"), "rb") as f:
        arena = f.read()
    if len(arena) != meta["arena_bytes"] or len(arena) != int(t["D.d_len"].numpy().astype(np.int64).sum()):
        raise CheckpointError(f"{d}: arena.bin is {len(arena)} bytes, expected {meta['arena_bytes']}")
    cols = {k: v for k, v in t.items() if k[:2] in ("S.", "P.", "D.", "G.", "T.")}
    host = {k: v for k, v in t.items() if k not in cols}
    return restore(hv, cols, host, arena, meta, verify="host", only=only)


def _host(cols: dict, host: dict, key: str) -> np.ndarray:
    """Host values of column ``key``: the host part's copy, else the column itself."""
    v = host.get("host." + key)
    if v is None:
        v = cols[key]
    return v.cpu().numpy() if isinstance(v, torch.Tensor) else np.asarray(v)


def restore(hv, cols: dict, host: dict, arena, meta: dict, verify: str = "host", only=None):
    """Write a columnar image (:func:`collect`'s ``cols``/``host``/``arena``/``meta``)
    into ``hv``'s store as new rows, registered lazily (:class:`RestoredBatch`).

    ``cols`` may be host tensors (checkpoint files) or tensors on the store device
    (a migration's received buffer: columns and ``arena`` are then written device
    to device, every row reference rewritten on the device).  ``verify``: ``"host"``
    re-verifies every chain and committed root over the bytes on the host before
    writing (checkpoint files), ``"device"`` runs K10/K09 over the written rows in
    place, ``"none"`` trusts the image."""
    from hypervisor.models import ConsistencyMode  # noqa: F401 - view construction needs it loaded

    st = hv._store
    sdev = st.device
    P = st.caps["P"]
    pcount_all = _host(cols, host, "S.s_pcount")
    if meta["participant_rows"] > P and len(pcount_all) and int(pcount_all.max()) > P:
        raise CheckpointError(f"checkpoint sessions have up to {int(pcount_all.max())} participants; "
                              f"store rows hold {P}")
    ids_col = _Col(host, "session_id")
    ids_all = ids_col.all()
    n_all = len(ids_all)
    doff_all, poff_all = host["off.delta"].numpy(), host["off.part"].numpy()
    goff_all, toff_all = host["off.saga"].numpy(), host["off.step"].numpy()
    dlen_all = _host(cols, host, "D.d_len").astype(np.int64)
    on_dev = isinstance(arena, torch.Tensor)
    # -- selection ----------------------------------------------------------------------
    if only is not None:
        if on_dev:
            raise ValueError("restore(only=...) reads a host image (checkpoint files)")
        want = set(only)
        sel = np.fromiter((s_ in want for s_ in ids_all), dtype=bool, count=n_all)
        si = np.flatnonzero(sel)
    else:
        si = np.arange(n_all, dtype=np.int64)
    n = len(si)
    dcnt = (doff_all[si + 1] - doff_all[si]).astype(np.int64)
    di = _ragged(doff_all[si], dcnt)
    pcnt = (poff_all[si + 1] - poff_all[si]).astype(np.int64)
    pi = _ragged(poff_all[si], pcnt)
    gcnt = (goff_all[si + 1] - goff_all[si]).astype(np.int64)
    gi = _ragged(goff_all[si], gcnt)
    tcnt = (toff_all[gi + 1] - toff_all[gi]).astype(np.int64)
    ti = _ragged(toff_all[gi], tcnt)
    doff = np.concatenate([[0], np.cumsum(dcnt)]).astype(np.int64)
    nd = len(di)

    def sub(v, ix):
        if only is None:
            return v
        return v[ix] if not isinstance(v, torch.Tensor) else v.index_select(0, torch.from_numpy(ix).to(v.device))

    grp = lambda pfx, ix: {k: sub(v, ix) for k, v in cols.items() if k.startswith(pfx)}  # noqa: E731
    S, Pc, D, G, Tt = grp("S.", si), grp("P.", pi), grp("D.", di), grp("G.", gi), grp("T.", ti)
    hs = lambda key, ix: sub(_host(cols, host, key), ix)  # noqa: E731 - host values of the selection
    dlen = dlen_all[di] if only is not None else dlen_all
    committed_h = hs("S.s_committed", si)
    # -- host K10 / K09 over the bytes about to be written -------------------------------------
    if verify == "host" and n:
        rec_all = np.zeros(len(dlen_all) + 1, dtype=np.int64)
        np.cumsum(dlen_all, out=rec_all[1:])
        rec_off = rec_all[di] if nd else np.zeros(0, np.int64)
        if only is not None and nd:  # the selected records, contiguous
            mv = memoryview(arena)
            blob = b"".join(mv[int(o):int(o) + int(ln)] for o, ln in zip(rec_off.tolist(), dlen.tolist()))
            rec_off = np.concatenate([[0], np.cumsum(dlen)[:-1]]).astype(np.int64)
        else:
            blob = arena
        commit_n = np.where(committed_h != 0, hs("S.s_commit_n", si), 0).astype(np.int32)
        dh = D["D.d_hash"].cpu().numpy() if isinstance(D["D.d_hash"], torch.Tensor) else D["D.d_hash"]
        sr = S["S.s_root"].cpu().numpy() if isinstance(S["S.s_root"], torch.Tensor) else S["S.s_root"]
        bad_c, bad_r = C.verify_chain_records(blob, rec_off, dlen, _as_np(D["D.d_hole"]).astype(np.int32),
                                              dh.astype(np.int32).view(np.uint32).reshape(-1),
                                              doff, sr.astype(np.int32).view(np.uint32).reshape(-1),
                                              commit_n, os.cpu_count() or 4)
        bc = np.frombuffer(bad_c, dtype=np.uint8)
        br = np.frombuffer(bad_r, dtype=np.uint8)
        if bc.any():
            k = int(np.flatnonzero(bc)[0])
            raise CheckpointError(f"session {ids_all[si[k]]}: audit chain fails re-verification "
                                  f"({int(bc.sum())} chain(s) in total)")
        if br.any():
            k = int(np.flatnonzero(br)[0])
            raise CheckpointError(f"session {ids_all[si[k]]}: Merkle root fails re-verification against its "
                                  f"commitment ({int(br.sum())} in total)")
        arena_sel = blob
    elif only is not None and nd:
        rec_all = np.concatenate([[0], np.cumsum(dlen_all)]).astype(np.int64)
        mv = memoryview(arena)
        arena_sel = b"".join(mv[int(rec_all[k]):int(rec_all[k] + dlen_all[k])] for k in di.tolist())
    else:
        arena_sel = arena
    # -- rows in the target store -------------------------------------------------------------
    agents = _Col(host, "agents").all()
    amap = np.asarray(st.agents.intern_many(agents), dtype=np.int64) if agents else np.zeros(0, np.int64)
    lut = torch.from_numpy(amap.astype(np.int32)).to(sdev) if len(amap) else None
    slots = st.alloc_many("S", n).astype(np.int64)
    if nd:
        rb, ob = st.reserve_deltas(dlen.astype(np.int32))
        drows = np.frombuffer(rb, dtype=np.int32).astype(np.int64)
        aoff = np.frombuffer(ob, dtype=np.int64).copy()
        if on_dev:
            from agent_hypervisor_amd.ops.store_views import move_records

            st.drain()
            move_records(st, torch.from_numpy(aoff).to(sdev), torch.from_numpy(dlen).to(sdev), arena_sel)
        else:
            st._c.write_records(aoff, dlen, arena_sel)
    else:
        drows = np.zeros(0, np.int64)
        aoff = np.zeros(0, np.int64)
    ng, nt = len(gi), len(ti)
    gslots = st.alloc_many("G", ng).astype(np.int64) if ng else np.zeros(0, np.int64)
    tslots = st.alloc_many("T", nt).astype(np.int64) if nt else np.zeros(0, np.int64)
    # -- columns with every row reference rewritten -------------------------------------------
    remap = lambda v: (lut.to(v.device)[v.to(torch.int64)] if isinstance(v, torch.Tensor)  # noqa: E731
                       else amap[v.astype(np.int64)].astype(np.int32)) if len(v) else v
    W: dict = {}
    for name in S_COLS:
        v = S[f"S.{name}"]
        W[name] = (slots, remap(v) if name == "s_creator" else v)
    for name, w in S_WIDE.items():
        W[name] = ((slots[:, None] * w + np.arange(w)[None, :]).reshape(-1), S[f"S.{name}"].reshape(-1))
    last = np.where(dcnt > 0, drows[np.maximum(doff[1:] - 1, 0)] if nd else -1, -1)
    W["s_dlast"] = (slots, last.astype(np.int32))
    W["s_proot_n"] = (slots, np.zeros(n, np.int32))
    kpos = np.arange(len(pi), dtype=np.int64) - np.repeat(np.concatenate([[0], np.cumsum(pcnt)[:-1]]), pcnt)
    prow = kpos * st.caps["S"] + np.repeat(slots, pcnt)  # participant-major (store.h prow), S after the allocs
    for name in P_COLS:
        v = Pc[f"P.{name}"]
        W[name] = (prow, remap(v) if name == "p_agent" else v)
    if nd:
        sess_of_d = np.repeat(np.arange(n, dtype=np.int64), dcnt)
        first = np.zeros(nd, dtype=bool)
        first[doff[:-1][dcnt > 0]] = True
        W["d_sess"] = (drows, slots[sess_of_d].astype(np.int32))
        W["d_prev"] = (drows, np.where(first, -1, np.roll(drows, 1)).astype(np.int32))
        W["d_off"] = (drows, aoff)
        for name in D_COLS:
            W[name] = (drows, D[f"D.{name}"])
        W["d_hash"] = ((drows[:, None] * 8 + np.arange(8)[None, :]).reshape(-1), D["D.d_hash"].reshape(-1))
    for name in G_COLS:
        W[name] = (gslots, G[f"G.{name}"])
    if nt:
        saga_of_t = np.repeat(np.arange(ng, dtype=np.int64), tcnt)
        W["t_saga"] = (tslots, gslots[saga_of_t].astype(np.int32))
    for name in T_COLS:
        W[name] = (tslots, Tt[f"T.{name}"])
    st.write_columns(W)
    if verify == "device" and n:
        cn = np.where(committed_h != 0, hs("S.s_commit_n", si), 0).astype(np.int64) if n else np.zeros(0, np.int64)
        try:
            _verify_on_device(st, slots, drows, doff, committed_h, ids_all, si, cn)
        except Exception:
            # nothing was registered: the rows written for the refused image go back
            st.release_many("S", slots)
            if nd:
                st.release_many("D", drows)
            if ng:
                st.release_many("G", gslots)
            if nt:
                st.release_many("T", tslots)
            raise
    # -- lazy registration ----------------------------------------------------------------------
    b = RestoredBatch()
    b.store = st
    b.ids = [ids_all[i] for i in si.tolist()] if only is not None else ids_all
    b.slots = slots.astype(np.int32)
    b.delta_off, b.drows, b.doff, b.dlen = doff, drows.astype(np.int32), aoff, dlen
    b.dhash = None if on_dev else (_as_np(D["D.d_hash"]).astype(np.int32).view(np.uint32).reshape(-1, 8) if nd
                                   else np.zeros((0, 8), np.uint32))
    b.dskip = host["sess.dskip"].numpy()[si]
    b.cfg_mode, b.cfg_maxdur, b.cfg_chain = host["sess.cfg_mode"].numpy()[si], host["sess.cfg_maxdur"].numpy()[si], \
        host["sess.cfg_chain"].numpy()[si]
    b.maxpart, b.minsig, b.audit = hs("S.s_maxpart", si), hs("S.s_minsig", si), hs("S.s_audit", si)
    b.creator = amap[hs("S.s_creator", si).astype(np.int64)] if n else np.zeros(0, np.int64)
    b.goff = np.concatenate([[0], np.cumsum(gcnt)]).astype(np.int64)
    b.gslots = gslots.astype(np.int32)
    b.toff = np.concatenate([[0], np.cumsum(tcnt)]).astype(np.int64)
    b.tslots = tslots.astype(np.int32)
    b.gid = _Col(host, "saga_id", mint="saga:").take(gi)
    b.gerr = _Col(host, "saga_error").take(gi)
    b.t_timeout = host["step.timeout"].numpy()[ti]
    b.tcols = {k: _Col(host, f"step.{k}", mint="step:" if k == "step_id" else None).take(ti)
               for k in ("step_id", "action_id", "agent_did", "execute_api", "undo_api", "error",
                         "execute_result", "compensation_result")}
    ex = meta.get("extras", {})
    pos_of = {int(i): k for k, i in enumerate(si.tolist())} if only is not None else None
    b.extras = {}
    for key, v in ex.items():
        i = int(key)
        j = i if pos_of is None else pos_of.get(i)
        if j is not None:
            b.extras[j] = v
    b.status = np.zeros(n, dtype=np.int32)
    b.built, b.released, b.dead = np.zeros(n, dtype=bool), np.zeros(n, dtype=bool), []
    b.index = dict(zip(b.ids, range(n)))
    b.views = {}
    b.committed = committed_h != 0 if n else np.zeros(0, dtype=bool)
    b._saga_ids = b._step_ids = None
    hv.commitment.register_batch(b)
    hv._sessions.add_batch(b, b.ids)
    hv.batched_sessions = max(int(getattr(hv, "batched_sessions", 0)), int(meta.get("batched_sessions", 0)))
    _restore_vouches(hv, meta["vouches"], None if only is None else set(only))
    _restore_commitments(hv, meta["commitments"], None if only is None else set(only))
    return hv


def _as_np(v) -> np.ndarray:
    return v.cpu().numpy() if isinstance(v, torch.Tensor) else v


def _verify_on_device(st, slots, drows, doff, committed, ids, si, commit_n=None) -> None:
    """K10 over the written rows (records re-hashed in the arena, parent links) and
    K09 over the committed chains, on the store's device.  A commitment covers the
    first ``s_commit_n`` deltas of its chain (the reference's ``capture`` has no state
    check, so a terminated session can gain deltas afterwards): the root is
    recomputed over that prefix, the same rule as the host path
    (``verify_chain_records(..., commit_n)``)."""
    from agent_hypervisor_amd.ops.store_views import store_roots, verify_store_chains

    chains = [drows[int(doff[i]):int(doff[i + 1])].tolist() for i in range(len(slots))]
    _, ok = verify_store_chains(st, chains)
    okh = ok.cpu().numpy()
    if not okh.all():
        k = int(np.flatnonzero(okh == 0)[0])
        raise CheckpointError(f"session {ids[si[k]]}: audit chain fails re-verification after the move")
    c = np.flatnonzero(committed != 0)
    if len(c):
        cut = [chains[i] if commit_n is None else chains[i][:int(commit_n[i])] for i in c.tolist()]
        roots = store_roots(st, cut).cpu().numpy()
        want = st.gather({"s_root": (slots[c][:, None] * 8 + np.arange(8)[None, :]).reshape(-1)})["s_root"]
        if not np.array_equal(roots.reshape(-1).astype(np.int64) & 0xFFFFFFFF,
                              want.astype(np.int64) & 0xFFFFFFFF):
            raise CheckpointError("Merkle root fails re-verification against its commitment after the move")


def _restore_vouches(hv, vouches: list, only: Optional[set]) -> None:
    from hypervisor import _device
    from hypervisor._clock import from_us

    st = hv._store
    ve = hv.vouching
    rows: dict = {}

    def put(c, i, v):
        ix, vs = rows.setdefault(c, ([], []))
        ix.append(i)
        vs.append(v)

    tails: dict = {}
    for v in vouches:
        if only is not None and v["session_id"] not in only:
            continue
        created = from_us(v["created_us"]) if v["created_us"] is not None else None
        expiry = from_us(v["expiry_us"]) if v["expiry_us"] is not None else None
        if v["linked"]:
            vs = st.liability_id(ve._tenant, v["session_id"])
            e = st.alloc("E")
            for c, val in (("e_voucher", st.agent_id(v["voucher_did"])), ("e_vouchee", st.agent_id(v["vouchee_did"])),
                           ("e_vsess", vs), ("e_next", -1), ("e_active", int(v["active"])),
                           ("e_bonded", float(v["bonded"])), ("e_pct", float(v["pct"])),
                           ("e_expiry", v["expiry_us"] if v["expiry_us"] is not None else -1),
                           ("e_released", int(v["released_us"])),
                           ("e_created", v["created_us"] if v["created_us"] is not None else 0)):
                put(c, e, val)
            if vs in tails:
                put("e_next", tails[vs], e)
            else:
                put("v_head", vs, e)
            tails[vs] = e
            put("v_tail", vs, e)
        else:
            e = -1
        rec = _device.DeviceVouchRecord(st, e, v["vouch_id"], v["voucher_did"], v["vouchee_did"], v["session_id"],
                                        v["pct"], v["bonded"], created, expiry, owner=ve)
        if e < 0:
            rec._freeze(int(v["active"]), int(v["released_us"]))
        else:
            ve._by_edge[e] = rec
        ve._by_id[rec.vouch_id] = rec
        ve._order.append(rec)
    if rows:
        st.write_rows(rows)


def _restore_commitments(hv, commits: list, only: Optional[set]) -> None:
    from hypervisor.audit.commitment import CommitmentRecord

    from agent_hypervisor_amd.runtime.checkpoint import _dt

    for c in commits:
        if only is not None and c["session_id"] not in only:
            continue
        hv.commitment._commitments[c["session_id"]] = CommitmentRecord(
            session_id=c["session_id"], merkle_root=c["merkle_root"], participant_dids=c["participant_dids"],
            delta_count=c["delta_count"], committed_at=_dt(c["committed_at"]),
            blockchain_tx_id=c["blockchain_tx_id"], committed_to=c["committed_to"])


# ---------------------------------------------------------------- lazy sessions


def _restored_batch_base():
    from agent_hypervisor_amd.models.store_pipeline import _Batch

    return _Batch


class RestoredBatch(_restored_batch_base()):
    """Sessions restored from a columnar checkpoint: rows written, views built on
    first use (:meth:`view`) from the rows and the restored descriptors.  Same
    session-table interface as the batched pipeline's ``_Batch``; a session may
    hold any number of sagas."""

    __slots__ = ("dskip", "cfg_mode", "cfg_maxdur", "cfg_chain", "maxpart", "minsig", "audit", "creator", "goff",
                 "toff", "gid", "gerr", "t_timeout", "tcols", "extras")

    def view(self, i: int):
        m = self.views.get(i)
        if m is None:
            from hypervisor.core import ManagedSession

            m = self.views[i] = ManagedSession(*self._materialize(i))
            self.built[i] = True
            _apply_extras(m, self.extras.get(i))
        return m

    def creator_did(self, i: int) -> str:
        return self.store.did(int(self.creator[i]))

    def rowref(self, i: int):
        from agent_hypervisor_amd.models.store_pipeline import _RowRef

        m = self.views.get(i)
        if m is not None:
            return m.sso
        return _RowRef(int(self.slots[i]), self.ids[i], self.creator_did(i))

    def rows(self, committed: bool = False) -> tuple:
        idx = np.fromiter(self.index.values(), dtype=np.int64, count=len(self.index))
        if committed:
            idx = idx[self.committed[idx]]
        did = self.store.did
        return self.slots[idx], [self.ids[i] for i in idx.tolist()], [did(int(a)) for a in self.creator[idx].tolist()]

    def release(self, idx: np.ndarray) -> None:
        idx = idx[~self.built[idx] & ~self.released[idx]]
        if not len(idx):
            return
        self.released[idx] = True
        st = self.store
        st.release_many("S", self.slots[idx])
        dr = _ragged(self.delta_off[idx], self.delta_off[idx + 1] - self.delta_off[idx])
        if len(dr):
            st.release_many("D", self.drows[dr])
        gr = _ragged(self.goff[idx], self.goff[idx + 1] - self.goff[idx])
        if len(gr):
            st.release_many("G", self.gslots[gr])
            tr = _ragged(self.toff[gr], self.toff[gr + 1] - self.toff[gr])
            if len(tr):
                st.release_many("T", self.tslots[tr])

    def saga_row_slots(self, idx) -> tuple:
        idx = np.asarray(idx, dtype=np.int64)
        gr = _ragged(self.goff[idx], self.goff[idx + 1] - self.goff[idx])
        tr = _ragged(self.toff[gr], self.toff[gr + 1] - self.toff[gr]) if len(gr) else np.zeros(0, np.int64)
        return self.gslots[gr].tolist(), self.tslots[tr].tolist()

    def saga_summaries(self, rows: dict, idx) -> list:
        from hypervisor._clock import from_us
        from hypervisor.saga.state_machine import SagaState, StepState

        gst, sst = list(SagaState), list(StepState)
        out, gk, tk = [], 0, 0
        tc = self.tcols
        for i in idx:
            for g in range(int(self.goff[i]), int(self.goff[i + 1])):
                steps = []
                for k in range(int(self.toff[g]), int(self.toff[g + 1])):
                    t0, t1 = int(rows["t_started"][tk]), int(rows["t_completed"][tk])
                    steps.append({"step_id": tc["step_id"][k], "action_id": tc["action_id"][k],
                                  "agent_did": tc["agent_did"][k], "state": sst[int(rows["t_state"][tk]) & 0xFF].value,
                                  "retry_count": int(rows["t_retry"][tk]), "error": tc["error"][k],
                                  "started_at": from_us(t0) if t0 else None,
                                      "completed_at": from_us(t1) if t1 else None})
                    tk += 1
                c1 = int(rows["g_completed"][gk])
                out.append({"saga_id": self.gid[g], "session_id": self.ids[i],
                            "state": gst[int(rows["g_state"][gk]) & 0xFF].value, "error": self.gerr[g],
                            "created_at": from_us(int(rows["g_created"][gk])),
                            "completed_at": from_us(c1) if c1 else None, "steps": steps})
                gk += 1
        return out

    def _materialize(self, i: int) -> tuple:
        from hypervisor import _device
        from hypervisor.audit.delta import VFSChange
        from hypervisor.models import ConsistencyMode, SessionConfig

        st = self.store
        sid = self.ids[i]
        slot = int(self.slots[i])
        md = float(self.cfg_maxdur[i])
        cfg = SessionConfig(consistency_mode=ConsistencyMode(_MODES[int(self.cfg_mode[i])]),
                            max_participants=int(self.maxpart[i]),
                            max_duration_seconds=None if math.isnan(md) else int(md),
                            min_sigma_eff=float(self.minsig[i]), enable_audit=bool(self.audit[i]),
                            enable_blockchain_commitment=bool(self.cfg_chain[i]))
        sso = _device.DeviceSession(st, cfg, self.creator_did(i), session_id=sid, slot=slot, create=False)
        de = _device.DeviceDeltaEngine(st, slot, sid, sso)
        d0, d1 = int(self.delta_off[i]), int(self.delta_off[i + 1])
        if d1 > d0:
            raw = st._c.payload_gather(self.doff[d0:d1], self.dlen[d0:d1])
            pos = 0
            prev = None
            skip = int(self.dskip[i])
            for g in range(d0, d1):
                ln = int(self.dlen[g])
                p = json.loads(raw[pos:pos + ln])
                pos += ln
                changes = [VFSChange(path=c["path"], operation=c["operation"], content_hash=c["content_hash"],
                                     previous_hash=c["previous_hash"]) for c in p["changes"]]
                v = _device.DeviceDelta(de, p["delta_id"], p["turn_id"], p["session_id"], p["agent_did"],
                                        datetime.fromisoformat(p["timestamp"]), changes, prev)
                h = "".join(f"{int(w):08x}" for w in self.dhash[g]) if self.dhash is not None else None
                v.__dict__.update(_didx=int(self.drows[g]), _poff=int(self.doff[g]), _plen=ln, _seq=-1, _dev_hash=h)
                de._rows.append(int(self.drows[g]))
                if g - d0 >= skip:
                    de._deltas.append(v)
                prev = v
        de._turn_counter = d1 - d0
        orch = _device.DeviceSagaOrchestrator(st, sso)
        tc = self.tcols
        for g in range(int(self.goff[i]), int(self.goff[i + 1])):
            saga = _device.DeviceSaga(st, int(self.gslots[g]), self.gid[g], sid)
            saga.error = self.gerr[g]
            for k in range(int(self.toff[g]), int(self.toff[g + 1])):
                mr = st.tables["t_maxretry"][int(self.tslots[k])]
                step = _device.DeviceSagaStep(
                    st, int(self.tslots[k]), step_id=tc["step_id"][k], action_id=tc["action_id"][k],
                    agent_did=tc["agent_did"][k], execute_api=tc["execute_api"][k], undo_api=tc["undo_api"][k],
                    timeout_seconds=_num(self.t_timeout[k]), max_retries=int(mr))
                step.__dict__.update(execute_result=json.loads(tc["execute_result"][k] or "null"),
                                     compensation_result=json.loads(tc["compensation_result"][k] or "null"),
                                     error=tc["error"][k])
                saga.steps.append(step)
            orch._sagas[saga.saga_id] = saga
        return sso, de, orch

    def __del__(self) -> None:
        try:
            self.release(np.arange(len(self.slots), dtype=np.int64))
        except Exception:  # noqa: BLE001 - interpreter shutdown
            pass


def _num(x: float):
    x = float(x)
    return int(x) if x.is_integer() else x


def _apply_extras(m, ex: Optional[dict]) -> None:
    if not ex:
        return
    from hypervisor.models import ActionDescriptor, ReversibilityLevel

    from agent_hypervisor_amd.runtime.checkpoint import _restore_vfs

    if "vfs" in ex:
        _restore_vfs(m.sso.vfs, ex["vfs"])
    for e in ex.get("reversibility", ()):
        m.reversibility.register(ActionDescriptor(
            action_id=e["action_id"], name=e["action_id"], execute_api=e["execute_api"], undo_api=e["undo_api"],
            reversibility=ReversibilityLevel(e["reversibility"]), undo_window_seconds=e["undo_window_seconds"],
            compensation_method=e["compensation_method"]))
        if not e["undo_api_healthy"]:
            m.reversibility.mark_undo_unhealthy(e["action_id"])


# ---------------------------------------------------------------- host-mode restore


def to_records(d: str, only=None) -> tuple:
    """The checkpoint as the per-session JSON records of the host format (so a
    host-mode hypervisor can load a device checkpoint): ``(records, vouches,
    commitments)`` in :func:`checkpoint.load_hypervisor`'s shapes."""
    from agent_hypervisor_amd.runtime.checkpoint import _iso
    from hypervisor._clock import from_us
    from hypervisor.models import SessionState
    from hypervisor.saga.state_machine import SagaState, StepState

    t, meta = read_tables(d)
    ids = _Col(t, "session_id").all()
    agents = _Col(t, "agents").all()
    with open(os.path.join(d, "arena.bin"), "rb") as f:
        arena = f.read()
    doff, poff, goff, toff = (t[k].numpy() for k in ("off.delta", "off.part", "off.saga", "off.step"))
    S = {k[2:]: v.numpy() for k, v in t.items() if k.startswith("S.")}
    Pc = {k[2:]: v.numpy() for k, v in t.items() if k.startswith("P.")}
    Dd = {k[2:]: v.numpy() for k, v in t.items() if k.startswith("D.")}
    G = {k[2:]: v.numpy() for k, v in t.items() if k.startswith("G.")}
    Tt = {k[2:]: v.numpy() for k, v in t.items() if k.startswith("T.")}
    gid, gerr = _Col(t, "saga_id", mint="saga:"), _Col(t, "saga_error")
    tc = {k: _Col(t, f"step.{k}", mint="step:" if k == "step_id" else None)
          for k in ("step_id", "action_id", "agent_did", "execute_api", "undo_api", "error", "execute_result",
                    "compensation_result")}
    rec_off = np.concatenate([[0], np.cumsum(Dd["d_len"].astype(np.int64))])
    states, sagas, steps = list(SessionState), list(SagaState), list(StepState)
    want = set(only) if only is not None else None
    iso = lambda us: _iso(from_us(int(us))) if us else None  # noqa: E731
    out = []
    for i, sid in enumerate(ids):
        if want is not None and sid not in want:
            continue
        md = float(t["sess.cfg_maxdur"][i])
        rec = {
            "session_id": sid, "creator_did": agents[int(S["s_creator"][i])],
            "state": states[int(S["s_state"][i])].value, "consistency_mode": _MODES[int(S["s_mode"][i])],
            "config": {"consistency_mode": _MODES[int(t["sess.cfg_mode"][i])],
                       "max_participants": int(S["s_maxpart"][i]),
                       "max_duration_seconds": None if math.isnan(md) else int(md),
                       "min_sigma_eff": float(S["s_minsig"][i]), "enable_audit": bool(S["s_audit"][i]),
                       "enable_blockchain_commitment": bool(t["sess.cfg_chain"][i])},
            "created_at": iso(S["s_created"][i]), "terminated_at": iso(S["s_terminated"][i]),
            "participants": [{"agent_did": agents[int(Pc["p_agent"][k])], "ring": int(Pc["p_ring"][k]),
                              "sigma_raw": float(Pc["p_sraw"][k]), "sigma_eff": float(Pc["p_seff"][k]),
                              "joined_at": iso(Pc["p_joined"][k]), "is_active": bool(Pc["p_active"][k] & 1)}
                             for k in range(int(poff[i]), int(poff[i + 1]))],
            "vfs": {"files": {}, "permissions": {}, "edits": []}, "reversibility": [],
            "turn_count": int(doff[i + 1] - doff[i]),
            "audit": [],
            "sagas": [],
        }
        ex = meta.get("extras", {}).get(str(i))
        if ex:
            rec["vfs"] = ex.get("vfs", rec["vfs"])
            rec["reversibility"] = ex.get("reversibility", [])
        skip = int(t["sess.dskip"][i])
        for k in range(int(doff[i]) + skip, int(doff[i + 1])):
            raw = arena[int(rec_off[k]):int(rec_off[k + 1])]
            rec["audit"].append({"payload": raw.decode("utf-8"),
                                 "delta_hash": "".join(f"{int(w) & 0xFFFFFFFF:08x}" for w in Dd["d_hash"][k])})
        for g in range(int(goff[i]), int(goff[i + 1])):
            rec["sagas"].append({
                "saga_id": gid[g], "session_id": sid, "state": sagas[int(G["g_state"][g])].value, "error": gerr[g],
                "created_at": iso(G["g_created"][g]), "completed_at": iso(G["g_completed"][g]),
                "steps": [{"step_id": tc["step_id"][k], "action_id": tc["action_id"][k],
                           "agent_did": tc["agent_did"][k], "execute_api": tc["execute_api"][k],
                           "undo_api": tc["undo_api"][k], "state": steps[int(Tt["t_state"][k])].value,
                           "error": tc["error"][k], "started_at": iso(Tt["t_started"][k]),
                           "completed_at": iso(Tt["t_completed"][k]),
                           "timeout_seconds": _num(t["step.timeout"][k]), "max_retries": int(Tt["t_maxretry"][k]),
                           "retry_count": int(Tt["t_retry"][k]),
                           "execute_result": json.loads(tc["execute_result"][k] or "null"),
                           "compensation_result": json.loads(tc["compensation_result"][k] or "null")}
                          for k in range(int(toff[g]), int(toff[g + 1]))]})
        out.append(rec)
    vouches = [{"vouch_id": v["vouch_id"], "voucher_did": v["voucher_did"], "vouchee_did": v["vouchee_did"],
                "session_id": v["session_id"], "bonded_sigma_pct": v["pct"], "bonded_amount": v["bonded"],
                "created_at": iso(v["created_us"]), "expiry": iso(v["expiry_us"]), "is_active": bool(v["active"]),
                "released_at": iso(v["released_us"]) if v["released_us"] and v["released_us"] > 0 else None}
               for v in meta["vouches"] if want is None or v["session_id"] in want]
    commits = list(meta["commitments"])
    for i, sid in enumerate(ids):
        if (want is None or sid in want) and int(S["s_committed"][i]):
            parts = [agents[int(Pc["p_agent"][k])] for k in range(int(poff[i]), int(poff[i + 1]))
                     if int(Pc["p_active"][k]) & 2]
            root = "".join(f"{int(w) & 0xFFFFFFFF:08x}" for w in S["s_root"][i])
            commits.append({"session_id": sid, "merkle_root": root, "participant_dids": parts,
                            "delta_count": int(S["s_commit_n"][i]), "committed_at": iso(S["s_committed"][i]),
                            "blockchain_tx_id": None, "committed_to": None})
    return out, vouches, commits
