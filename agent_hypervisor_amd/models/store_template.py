"""The reference pipeline for a whole batch of sessions, over the store's rows.

One launch of ``store_template_kernel`` (``csrc/hip/store_template.hip``, body in
``csrc/include/ahv/store_template.h``) runs the reference benchmark's pipeline
(``benchmarks/bench_hypervisor.py:217-239``: create → join with the σ ring gate →
activate → D audit deltas → saga step → terminate with Merkle root) for every
session of the batch, one lane per session, and writes *store* rows — session,
participant, delta (with its canonical-JSON record in the payload arena), saga
and step rows — exactly as the per-call API's commands would.  There is one
device state: the sessions are ordinary sessions of the hypervisor afterwards
(``hv.get_session``, terminate, ``verify_audit`` over the arena in place,
checkpoints), reference ``core.py:92-103``.

Two ways in:

* :func:`run` / ``Hypervisor.pipeline_batch(n)`` — one batch, registered lazily
  with the hypervisor (no per-session Python objects until a session is used);
* :class:`TemplatePipeline` — rows allocated once and re-run step after step
  (``reset`` frees them in place on the stream): the headline step of
  ``bench.py``.  Session ids are minted on the device from a counter
  (``uuid4_words(seed, id_base + i)``), so a step costs no host work per session.
"""

from __future__ import annotations

import os
from typing import Optional, Sequence

import numpy as np
import torch

from agent_hypervisor_amd._native import C
from agent_hypervisor_amd.utils.stats import SpreadCounters

REFERENCE_CHANGES = (("/f{i}", "add", "h{i}"),)  # bench_hypervisor.py:232-233

# canonical-JSON literal lengths (csrc/include/ahv/canon_json.h) of one record
_K = dict(open_agent=14, changes=14, ch_open=18, ch_op=15, ch_path=10, ch_prev=19, ch_close=1, ch_sep=2,
          delta_id=16, delta_pfx=7, parent=17, session=16, ts=15, turn=13, close=1)


class AgentSet:
    """Agents a template batch draws from: their store ids (participant rows), pool
    ids (rendered DIDs) and σ_raw, as device arrays (index = agent number)."""

    def __init__(self, store, dids: Sequence[str], sigmas) -> None:
        dev = store.device
        self.store = store
        self.dids = list(dids)
        ids = store.agents.intern_many(self.dids)
        pools = store.pool.intern_many(self.dids)
        self.agent_id = torch.as_tensor(np.asarray(ids, dtype=np.int32)).to(dev)
        self.agent_pool = torch.as_tensor(np.asarray(pools, dtype=np.int32)).to(dev)
        self.sigma = torch.as_tensor(np.asarray(sigmas, dtype=np.float64)).to(dev)
        if self.sigma.numel() != len(self.dids):
            raise ValueError("one σ per agent")
        self.max_did = max((len(store.pool.escaped(p)) for p in pools), default=0)

    @property
    def count(self) -> int:
        return len(self.dids)

    @classmethod
    def synthetic(cls, store, n: int, seed: int = 0, prefix: str = "did:mesh:agent-") -> "AgentSet":
        """``n`` agents with random-init σ ~ U[0, 1) (the BASELINE synthetic population)."""
        g = torch.Generator().manual_seed(seed)
        sig = torch.rand(n, generator=g, dtype=torch.float64).numpy()
        return cls(store, [f"{prefix}{k}" for k in range(n)], sig)


def _record_cap(store, changes_rows, turn: int, max_did: int) -> int:
    """Arena bytes reserved for a record of ``turn``: the padded SHA-256 message of
    the longest possible record (longest DID, microsecond timestamp)."""
    k = _K
    n = k["open_agent"] + max_did + 2 + k["changes"]
    for j, (p, o, h, ph) in enumerate(changes_rows):
        esc = lambda i: 4 if i < 0 else len(store.pool.escaped(i)) + 2  # noqa: E731
        n += (k["ch_sep"] if j else 0) + k["ch_open"] + esc(h) + k["ch_op"] + esc(o) + k["ch_path"] + esc(p)
        n += k["ch_prev"] + esc(ph) + k["ch_close"]
    digits = len(str(turn))
    n += k["delta_id"] + k["delta_pfx"] + digits + 1 + k["parent"] + (66 if turn > 1 else 4)
    n += k["session"] + 46 + k["ts"] + 34 + k["turn"] + digits + k["close"]
    return (n + 9 + 63) & ~63


class TemplatePipeline:
    """Store rows + device arguments for ``n`` sessions of one pipeline spec.

    ``launch`` runs the whole pipeline over the rows (they must be free: the
    first launch after construction, or after :meth:`reset`); each launch mints
    new session ids (``id_base`` advances by ``n``)."""

    def __init__(self, store, n: int, agents: AgentSet, deltas: int = 3, changes=REFERENCE_CHANGES,
                 config=None, creator_did: str = "did:mesh:admin", gc_retention_days: int = 90,
                 seed: Optional[int] = None) -> None:
        from hypervisor.models import SessionConfig

        if not 0 <= deltas <= 8:
            raise ValueError("deltas must be in [0, 8]")
        if not 0 <= len(changes) <= 4:
            raise ValueError("at most 4 changes per delta")
        cfg = config or SessionConfig()
        st = self.store = store
        dev = st.device
        self.n, self.deltas, self.agents, self.config = n, deltas, agents, cfg
        self.changes = tuple(changes)
        self.creator_did = creator_did
        pool = st.pool
        rows = []
        for d in range(deltas):
            for spec in changes:
                p, o, h = spec[0], spec[1], spec[2]
                ph = spec[3] if len(spec) > 3 else None
                rows.append([pool.intern(p.format(i=d)), pool.intern(o.format(i=d)),
                             pool.intern(h.format(i=d)) if h is not None else -1,
                             pool.intern(ph.format(i=d)) if ph is not None else -1])
        nch = len(changes)
        caps = [_record_cap(st, rows[d * nch:(d + 1) * nch], d + 1, agents.max_did) for d in range(deltas)]
        self.max_rec = max(caps) if caps else 0  # the cooperative small-batch kernel needs ≤ 512 (8 blocks)
        self.slots = st.alloc_many("S", n)
        self.gslots = st.alloc_many("G", n)
        self.tslots = st.alloc_many("T", n)
        if deltas:
            drows, doff = st.reserve_deltas(np.tile(np.asarray(caps, dtype=np.int32), n))
            self.drows = np.frombuffer(drows, dtype=np.int32)
            self.doff = np.frombuffer(doff, dtype=np.int64)
        else:
            self.drows = np.zeros(0, dtype=np.int32)
            self.doff = np.zeros(0, dtype=np.int64)
        T = lambda a: torch.from_numpy(np.array(a, copy=True)).to(dev)  # noqa: E731
        self.tens = {
            "slot": T(self.slots), "gslot": T(self.gslots), "tslot": T(self.tslots),
            "drow": T(self.drows) if deltas else torch.zeros(1, dtype=torch.int32, device=dev),
            "doff": T(self.doff) if deltas else torch.zeros(1, dtype=torch.int64, device=dev),
            "changes": torch.tensor(rows or [[0, 0, 0, 0]], dtype=torch.int32).to(dev),
            "status": torch.zeros(n, dtype=torch.int32, device=dev),
        }
        # each delta's changes fragment (`, "changes": [...], ..., "parent_hash": `) is the
        # same for every session: rendered once here, copied by the kernel through the
        # scalar cache (AHV_TEMPLATE_FRAG=0: rendered per session and pass from the pool)
        if deltas and os.environ.get("AHV_TEMPLATE_FRAG", "1") != "0":
            words, offs, lens = [], [], []
            for d in range(deltas):
                b = C.render_fragment(pool._pool, rows[d * nch:(d + 1) * nch], d + 1, d > 0)
                offs.append(sum(len(x) for x in words))
                lens.append(len(b))
                words.append(np.frombuffer(b + b"\0" * (-len(b) % 4), dtype=">u4").astype(np.uint32))
            self.tens["frag"] = T(np.concatenate(words).view(np.int32))
            self.tens["frag_off"] = T(np.asarray(offs, dtype=np.int32))
            self.tens["frag_len"] = T(np.asarray(lens, dtype=np.int32))
        self._slots64 = {k: self.tens[k].to(torch.int64) for k in ("slot", "gslot", "tslot")}
        self.seed = int(seed if seed is not None else st.seed) & ((1 << 63) - 1)
        self._own_seed = seed is not None
        self.t0 = 0
        self.creator = st.agent_id(creator_did)
        self.gc_retention_us = int(gc_retention_days) * 86_400 * 1_000_000
        self._spread = SpreadCounters(6, dev)

    def reset(self) -> None:
        """Free the batch's session / saga / step rows in place, on the stream (so
        the next :meth:`launch` runs the whole pipeline over them again)."""
        t = self.store.tables
        t["s_state"].index_fill_(0, self._slots64["slot"], 255)  # kFree8
        t["g_state"].index_fill_(0, self._slots64["gslot"], 255)
        t["t_state"].index_fill_(0, self._slots64["tslot"], 255)

    def launch(self, session_agent: torch.Tensor, t0: Optional[int] = None, stats: Optional[torch.Tensor] = None,
               sync: bool = True, variant: Optional[tuple] = None, extra: Optional[dict] = None) -> tuple:
        """Run the pipeline for every session; ``session_agent`` = int32 [n] agent
        numbers (which agent joins and captures in each session).  ``stats``
        (int64[6]) accumulates sessions / ok / participants / deltas / commits /
        archived.  Returns ``(id_base, t0)`` of this launch.  ``sync``: make the
        store worker's pending writes visible first and its view of the new rows
        after (off in a benchmark's steady state, where nothing else writes).
        ``variant``: ``(waves, small)`` kernel selection for this launch (default:
        ``AHV_TEMPLATE_WAVES`` / ``AHV_TEMPLATE_SMALL``; ``small`` is the largest
        batch that takes the one-pass ``<1,6>`` kernel)."""
        from hypervisor._clock import now_us

        st = self.store
        dev = st.device
        if session_agent.numel() != self.n:
            raise ValueError("one agent per session")
        sa = session_agent.to(dev, torch.int32).contiguous()
        if sa.numel() and sync:
            lo, hi = int(sa.min()), int(sa.max())
            if lo < 0 or hi >= self.agents.count:
                raise ValueError(f"agent numbers out of range [0, {self.agents.count})")
        pb, po, pl = st.pool.device_view(dev)
        t0 = int(t0 if t0 is not None else now_us())
        # a fresh counter range for this launch's ids: launches of every template batch
        # on one store share the store's generator, so their ids never collide
        id_base = st.reserve_ids(self.n) if not self._own_seed else self._next_own(self.n)
        cfg = self.config
        tens = self.tens
        args = {
            "n": self.n, "slot": tens["slot"].data_ptr(), "gslot": tens["gslot"].data_ptr(),
            "tslot": tens["tslot"].data_ptr(), "drow": tens["drow"].data_ptr(), "doff": tens["doff"].data_ptr(),
            "session_agent": sa.data_ptr(), "agent_id": self.agents.agent_id.data_ptr(),
            "agent_pool": self.agents.agent_pool.data_ptr(), "agent_sigma": self.agents.sigma.data_ptr(),
            "changes": tens["changes"].data_ptr(), "pool_bytes": pb.data_ptr(), "pool_off": po.data_ptr(),
            "pool_len": pl.data_ptr(), "deltas": self.deltas, "nch": len(self.changes), "creator": self.creator,
            "maxpart": int(cfg.max_participants), "minsig": float(cfg.min_sigma_eff),
            "audit": int(bool(cfg.enable_audit)), "t0": t0, "seed": self.seed, "id_base": id_base,
            "gc_retention_us": self.gc_retention_us, "status": tens["status"].data_ptr(),
            "stats": self._spread.begin().data_ptr() if stats is not None else None,
            "max_rec": self.max_rec,
        }
        if "frag" in tens:
            args.update(frag=tens["frag"].data_ptr(), frag_off=tens["frag_off"].data_ptr(),
                        frag_len=tens["frag_len"].data_ptr())
        if variant is not None:
            args["waves"], args["small"] = int(variant[0]), int(variant[1])
        if extra:  # measurement knobs (e.g. "phase_ticks": a uint64 device pointer)
            args.update(extra)
        cuda = dev.type == "cuda"
        if cuda:
            if sync:
                st.drain()
                st.flush()  # frees / creates the worker wrote are visible to the kernel
            st._c.run_template(args, torch.cuda.current_stream(dev).cuda_stream)
        else:
            st._c.run_template(args, 0)
        if stats is not None:
            self._spread.add_into(stats)
        if cuda and sync:
            torch.cuda.synchronize(dev)
            st.acquire()  # the worker sees the batch's rows
        self.t0 = t0
        self.last_id_base = id_base
        self._keep = sa  # the launch reads it asynchronously
        return id_base, t0

    def _next_own(self, n: int) -> int:
        b = getattr(self, "_own_base", 0)
        self._own_base = b + n
        return b

    def session_ids(self, id_base: int) -> list:
        """The session ids a launch with ``id_base`` minted (host formatting of the
        device's counter-based uuid4 words)."""
        return C.uuids_from_counters(self.seed, id_base, self.n, "session:")


class _TemplateSpecs:
    """Per-session :class:`PipelineSpec` view of a template batch (built on demand:
    only the sessions whose views are materialised ever need one)."""

    def __init__(self, tp: TemplatePipeline, agent_idx: np.ndarray) -> None:
        self.tp = tp
        self.agent_idx = agent_idx
        self.sigma = tp.agents.sigma.cpu().numpy() if agent_idx is not None else None
        self._cache: dict = {}

    def __len__(self) -> int:
        return self.tp.n

    def __getitem__(self, i: int):
        from agent_hypervisor_amd.models.store_pipeline import PipelineSpec

        a = int(self.agent_idx[i])
        sp = self._cache.get(a)
        if sp is None:
            tp = self.tp
            did = tp.agents.dids[a]
            deltas = tuple((did, tuple(tuple(x.format(i=d) if x is not None else None for x in c) for c in tp.changes))
                           for d in range(tp.deltas))
            sp = PipelineSpec(joins=((did, float(self.sigma[a])),), deltas=deltas,
                              steps=(("action", did, "/api/action", None, 0, 0),), config=tp.config,
                              creator_did=tp.creator_did)
            if len(self._cache) < 4096:
                self._cache[a] = sp
        return sp


def run(hv, n: int, agents: Optional[AgentSet] = None, session_agent=None, deltas: int = 3,
        changes=REFERENCE_CHANGES, now_us: Optional[int] = None, config=None,
        creator_did: str = "did:mesh:admin", variant: Optional[tuple] = None):
    """One template batch of ``n`` sessions registered with ``hv`` (lazily): returns
    a :class:`~agent_hypervisor_amd.models.store_pipeline.PipelineRun`.  Without
    ``agents``, a synthetic population the size of the batch (random-init σ) is
    registered once per store; ``session_agent`` defaults to agent ``i % count``."""
    from agent_hypervisor_amd.models import store_pipeline as SP

    st = hv._store
    if st is None:
        raise RuntimeError("pipeline_batch needs a device-backed Hypervisor (device='cuda' or 'cpu')")
    if agents is None:
        agents = getattr(st, "_template_agents", None)
        if agents is None or agents.count < min(n, 1 << 20):
            agents = st._template_agents = AgentSet.synthetic(st, max(min(n, 1 << 20), 1024))
    tp = TemplatePipeline(st, n, agents, deltas=deltas, changes=changes, config=config, creator_did=creator_did,
                          gc_retention_days=int(hv.gc.policy.delta_retention_days))
    if session_agent is None:
        session_agent = torch.arange(n, dtype=torch.int32) % agents.count
    sa = torch.as_tensor(session_agent, dtype=torch.int32)
    id_base, t0 = tp.launch(sa, t0=now_us, variant=variant)
    ids = tp.session_ids(id_base)
    # what the lazy views need, in one copy each (the batched API's finish step)
    status = tp.tens["status"].cpu().numpy()
    nd = len(tp.drows)
    gath = st.gather({"d_len": tp.drows, "d_hash": (tp.drows.astype(np.int64)[:, None] * 8
                                                     + np.arange(8, dtype=np.int64)[None, :]).reshape(-1)}) \
        if nd else {"d_len": np.zeros(0, np.int32), "d_hash": np.zeros(0, np.int32)}
    committed = np.zeros(0, dtype=np.int64)
    flat = ""
    if deltas and (config is None or config.enable_audit):
        cs = tp.slots.astype(np.int64)
        gg = st.gather({"s_root": (cs[:, None] * 8 + np.arange(8, dtype=np.int64)[None, :]).reshape(-1),
                        "s_committed": cs})
        keep = np.flatnonzero(gg["s_committed"])
        committed = keep.astype(np.int64)
        flat = gg["s_root"].astype(np.uint32).reshape(-1, 8)[keep].byteswap().tobytes().hex()
    b = SP._Batch()
    b.store, b.specs, b.shared, b.ids, b.slots, b.t0 = st, _TemplateSpecs(tp, sa.numpy()), False, ids, tp.slots, t0
    b.doff, b.drows = tp.doff, tp.drows
    b.dlen = gath["d_len"].astype(np.int64)
    b.dhash = gath["d_hash"].astype(np.uint32).reshape(-1, 8) if nd else np.zeros((0, 8), np.uint32)
    b.delta_off = np.arange(0, (n + 1) * deltas, deltas, dtype=np.int32) if deltas else np.zeros(n + 1, np.int32)
    b.gslots, b.tslots = tp.gslots, tp.tslots
    b.step_off = np.arange(n + 1, dtype=np.int32)
    b.status, b.built, b.released, b.dead = status, np.zeros(n, dtype=bool), np.zeros(n, dtype=bool), []
    b._saga_ids = b._step_ids = None
    b.reserve_saga_ids()
    SP.register_lazy(hv, b, status, committed)
    out = SP.PipelineRun(session_ids=ids, status=status, join_rings=np.zeros(0, np.uint8),
                         join_codes=np.zeros(0, np.uint8))
    out._roots = (committed, flat)
    return out


def reference_records(session_id: str, did: str, t0: int, deltas: int, changes=REFERENCE_CHANGES) -> list:
    """The canonical-JSON records the scalar API renders for one template session
    (reference ``audit/delta.py:41-64``): delta k at ``t0 + 1 + k`` µs, chained."""
    import hashlib

    from hypervisor._clock import from_us
    from hypervisor.audit.delta import SemanticDelta, VFSChange, _payload_json

    out, parent = [], None
    for k in range(deltas):
        chs = []
        for spec in changes:
            p, o, h = spec[0], spec[1], spec[2]
            ph = spec[3] if len(spec) > 3 else None
            chs.append(VFSChange(path=p.format(i=k), operation=o.format(i=k),
                                 content_hash=h.format(i=k) if h is not None else None,
                                 previous_hash=ph.format(i=k) if ph is not None else None))
        d = SemanticDelta(delta_id=f"delta:{k + 1}", turn_id=k + 1, session_id=session_id, agent_did=did,
                          timestamp=from_us(t0 + 1 + k), changes=chs, parent_hash=parent)
        raw = _payload_json(d).encode()
        out.append(raw)
        parent = hashlib.sha256(raw).hexdigest()
    return out


def reference_merkle(leaves: list) -> Optional[str]:
    """Reference ``compute_merkle_root`` (``audit/delta.py:117-134``) over hex leaves."""
    import hashlib

    if not leaves:
        return None
    level = list(leaves)
    while len(level) > 1:
        if len(level) % 2:
            level.append(level[-1])
        level = [hashlib.sha256((level[k] + level[k + 1]).encode()).hexdigest() for k in range(0, len(level), 2)]
    return level[0]


def check_sessions(tp: TemplatePipeline, id_base: int, t0: int, session_agent, idx) -> int:
    """Oracle check of sessions ``idx`` of one :meth:`TemplatePipeline.launch`
    (``id_base``, ``t0`` and the ``session_agent`` it was given) against the host:
    every arena record equals the scalar renderer's bytes, every ``d_hash`` is
    hashlib's SHA-256 of it, ``s_head`` is the last digest and ``s_root`` the
    reference Merkle root.  Raises ``AssertionError`` naming the first mismatch;
    returns the number of sessions checked."""
    st = tp.store
    idx = np.asarray(idx, dtype=np.int64)
    if not len(idx):
        return 0
    D = tp.deltas
    sa = torch.as_tensor(session_agent).to("cpu", torch.int64).numpy()[idx]
    slots = tp.slots[idx].astype(np.int64)
    rows = tp.drows.reshape(-1, D)[idx].astype(np.int64) if D else np.zeros((len(idx), 0), np.int64)
    offs = tp.doff.reshape(-1, D)[idx] if D else np.zeros((len(idx), 0), np.int64)
    w8 = np.arange(8, dtype=np.int64)
    flat = rows.reshape(-1)
    g = st.gather({"d_len": flat, "d_hash": (flat[:, None] * 8 + w8).reshape(-1),
                   "s_head": (slots[:, None] * 8 + w8).reshape(-1), "s_root": (slots[:, None] * 8 + w8).reshape(-1),
                   "s_committed": slots, "s_state": slots})
    lens = g["d_len"].astype(np.int64).reshape(len(idx), D)
    hx = lambda w: w.astype(np.uint32).byteswap().tobytes().hex()  # noqa: E731 - 8 digest words → hex
    dh = g["d_hash"].reshape(len(idx), D, 8)
    heads, roots = g["s_head"].reshape(-1, 8), g["s_root"].reshape(-1, 8)
    audit = bool(tp.config.enable_audit) and D > 0
    for k, i in enumerate(idx.tolist()):
        sid = C.uuids_from_counters(tp.seed, id_base + i, 1, "session:")[0]
        did = tp.agents.dids[int(sa[k])]
        recs = reference_records(sid, did, t0, D, tp.changes)
        got = st._c.payload_gather(offs[k].astype(np.int64), lens[k]) if D else b""
        assert got == b"".join(recs), f"session {i} ({sid}): arena records differ from the scalar renderer"
        import hashlib

        leaves = [hashlib.sha256(r).hexdigest() for r in recs]
        dev_leaves = [hx(dh[k, d]) for d in range(D)]
        assert dev_leaves == leaves, f"session {i}: d_hash differs from hashlib"
        if D:
            assert hx(heads[k]) == leaves[-1], f"session {i}: s_head is not the chain's last digest"
        if audit:
            assert int(g["s_committed"][k]) != 0, f"session {i}: not committed"
            assert hx(roots[k]) == reference_merkle(leaves), f"session {i}: s_root is not the reference Merkle root"
    return len(idx)
