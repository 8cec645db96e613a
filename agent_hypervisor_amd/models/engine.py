"""GovernanceEngine: the batched governance pipeline as a standalone engine.

It runs the reference benchmark's full pipeline (bench_hypervisor.py:217-239)

    create → join (σ ring gate) → activate → D × audit capture (canonical JSON +
    SHA-256 Merkle chain) → saga create/add/execute → terminate (Merkle root,
    commitment, GC, archive)

for a whole batch of sessions in one gfx950 launch — the template pipeline
kernel (``csrc/hip/store_template.hip``) — over the rows of a *store*
(:class:`~agent_hypervisor_amd.models.store.GovernanceStore`): session,
participant, delta (with its canonical-JSON record in the payload arena), saga
and step rows, the same layout and kernel body the device-backed
``Hypervisor`` uses (one representation of session state; there is no separate
engine table any more).  The engine owns its store outright and uses it as a
ring: batch k takes the next ``n`` rows (mod capacity) and evicts whatever
sessions they held, which is what a steady-state batch generator (hipGraph
replay, :class:`agent_hypervisor_amd.runtime.graphs.PipelineGraph`) needs.

Ids (session / saga / step uuid4) come from a counter-based generator (three per
session; the session's are minted on device into ``s_uuid``), timestamps from one
injected ``now_us`` per batch (N09), and every digest is byte-identical to what
the scalar path computes for the same ids and timestamps
(``tests/test_engine_host.py``, ``tests/test_gpu_pipeline.py``).

``engine.sessions`` keeps the engine's historical column names as views over
the store's columns (``sess_state`` → ``s_state``, ``delta_hash`` → ``d_hash``
as [capacity, dmax, 8], ...).

Multi-GPU: one engine per rank; sessions are sharded by rank (P01), see
:mod:`agent_hypervisor_amd.parallel.directory`.
"""

from __future__ import annotations

import os
import time
from dataclasses import dataclass
from typing import Optional, Sequence

import numpy as np
import torch

from agent_hypervisor_amd._native import C
from agent_hypervisor_amd.models.store import GovernanceStore
from agent_hypervisor_amd.models.store_template import _record_cap
from agent_hypervisor_amd.ops import pipeline as _pipeline_op
from agent_hypervisor_amd.utils.stats import SpreadCounters
from hypervisor import _clock
from hypervisor.config import RUNTIME

REFERENCE_CHANGES = [("/f{i}", "add", "h{i}")]  # bench_hypervisor.py:232-233


def resolve_device(device: Optional[str]) -> torch.device:
    d = torch.device(device or RUNTIME.device)
    if d.type == "cuda" and not torch.cuda.is_available():
        raise RuntimeError(
            "GovernanceEngine requested a HIP device but torch.cuda.is_available() is False; "
            "pass device='cpu' explicitly to run the host twin"
        )
    if d.type == "cuda" and d.index is None:
        d = torch.device("cuda", torch.cuda.current_device())  # tensors report an explicit index
    return d


def _u32_hex(words: torch.Tensor) -> str:
    return "".join(f"{int(w) & 0xFFFFFFFF:08x}" for w in words.tolist())


def _uuid_str(words: torch.Tensor) -> str:
    h = _u32_hex(words)
    return f"{h[:8]}-{h[8:12]}-{h[12:16]}-{h[16:20]}-{h[20:]}"


class EngineSessions:
    """The engine's session columns under their historical names: views over the
    store's tables (no copy; the engine's store never grows)."""

    _MAP = {  # name → (store column, row shape)
        "sess_uuid": ("s_uuid", 4), "sess_state": ("s_state", None), "sess_mode": ("s_mode", None),
        "sess_creator": ("s_creator", None), "sess_created_us": ("s_created", None),
        "sess_terminated_us": ("s_terminated", None), "part_count": ("s_pcount", None),
        "part_agent": ("p_agent", "P"), "part_ring": ("p_ring", "P"), "part_sigma_raw": ("p_sraw", "P"),
        "part_sigma_eff": ("p_seff", "P"), "part_joined_us": ("p_joined", "P"), "delta_count": ("s_dcount", None),
        "merkle_root": ("s_root", 8), "saga_state": ("g_state", None), "step_state": ("t_state", None),
        "step_started_us": ("t_started", None), "step_completed_us": ("t_completed", None),
        "committed_at_us": ("s_committed", None), "gc_retained": ("s_retained", None),
        "bonds_released": ("s_released", None),
    }
    COLUMNS = tuple(_MAP) + ("delta_hash", "status")

    def __init__(self, store: GovernanceStore, capacity: int, dmax: int, status: torch.Tensor) -> None:
        self.capacity, self.dmax = capacity, dmax
        t, P = store.tables, store.caps["P"]
        for name, (col, shape) in self._MAP.items():
            x = t[col]
            if shape == "P":  # participant-major columns (store.h prow): [P][S] → a [cap, P] view
                x = x[: P * store.caps["S"]].view(P, store.caps["S"])[:, :capacity].t()
            elif shape is not None:
                x = x[: capacity * shape].view(capacity, shape)
            else:
                x = x[:capacity]
            setattr(self, name, x)
        self.delta_hash = t["d_hash"][: capacity * dmax * 8].view(capacity, dmax, 8)
        self.status = status


class AgentRegistry:
    """Agents a batch draws from (index = agent number): σ_raw, the pool id of the
    DID (rendered into records) and the store agent id (participant rows)."""

    def __init__(self, store: GovernanceStore, capacity: int) -> None:
        dev = store.device
        self.store = store
        self.capacity = capacity
        self.count = 0
        self.sigma = torch.zeros(capacity, dtype=torch.float64, device=dev)
        self.did = torch.zeros(capacity, dtype=torch.int32, device=dev)  # pool ids
        self.store_id = torch.zeros(capacity, dtype=torch.int32, device=dev)
        self.max_did = 0

    def add(self, dids: Sequence[str], sigmas) -> torch.Tensor:
        dids = list(dids)
        k = len(dids)
        if self.count + k > self.capacity:
            raise ValueError(f"agent table full ({self.capacity})")
        st = self.store
        pools = st.pool.intern_many(dids)
        ids = st.agents.intern_many(dids)
        s = torch.as_tensor(sigmas, dtype=torch.float64)
        if s.numel() != k:
            raise ValueError("one σ per agent")
        lo = self.count
        self.sigma[lo:lo + k] = s.to(self.sigma.device)
        self.did[lo:lo + k] = torch.as_tensor(np.asarray(pools, dtype=np.int32)).to(self.did.device)
        self.store_id[lo:lo + k] = torch.as_tensor(np.asarray(ids, dtype=np.int32)).to(self.did.device)
        self.max_did = max([self.max_did] + [len(st.pool.escaped(p)) for p in set(pools)])
        self.count += k
        return torch.arange(lo, lo + k, dtype=torch.int32)


@dataclass
class PipelineBatch:
    """Handle on the rows one ``run_pipeline`` call wrote."""

    engine: "GovernanceEngine"
    slot_base: int
    n: int
    id_base: int
    now_us: int
    deltas: int
    change_specs: list
    agent_ids: torch.Tensor

    def slots(self) -> torch.Tensor:
        cap = self.engine.sessions.capacity
        return (torch.arange(self.n, device=self.engine.device) + self.slot_base) % cap

    def _slot(self, i: int) -> int:
        if not 0 <= i < self.n:
            raise IndexError(i)
        return (self.slot_base + i) % self.engine.sessions.capacity

    def session_id(self, i: int) -> str:
        return "session:" + _uuid_str(self.engine.sessions.sess_uuid[self._slot(i)].cpu())

    def saga_id(self, i: int) -> str:
        self._slot(i)
        return C.uuid_from_counter(self.engine.seed, self.id_base + 3 * i + 1, "saga:")

    def step_id(self, i: int) -> str:
        self._slot(i)
        return C.uuid_from_counter(self.engine.seed, self.id_base + 3 * i + 2, "step:")

    def merkle_root_hex(self, i: int) -> str:
        return _u32_hex(self.engine.sessions.merkle_root[self._slot(i)].cpu())

    def delta_hash_hex(self, i: int, d: int) -> str:
        return _u32_hex(self.engine.sessions.delta_hash[self._slot(i), d].cpu())

    def roots(self) -> torch.Tensor:
        return self.engine.sessions.merkle_root.index_select(0, self.slots())

    def status(self) -> torch.Tensor:
        return self.engine.sessions.status.index_select(0, self.slots())

    def record(self, i: int, d: int) -> bytes:
        """The canonical-JSON record of delta ``d`` of session ``i`` as the kernel
        wrote it into the store's payload arena (the exact hashed bytes)."""
        eng = self.engine
        dr = self._slot(i) * eng.sessions.dmax + d
        st = eng.store
        off = int(st.tables["d_off"][dr])
        ln = int(st.tables["d_len"][dr])
        return st.payload(off, ln)

    def materialize(self, i: int):
        """Rebuild the scalar-API view (``ManagedSession``) of one session.

        The returned session's delta engine re-hashes on the host, so
        ``verify_chain()`` and ``compute_merkle_root()`` independently check the
        device results.
        """
        from hypervisor.audit.delta import SemanticDelta, VFSChange
        from hypervisor.core import ManagedSession
        from hypervisor.models import ExecutionRing, SessionConfig, SessionParticipant, SessionState
        from hypervisor.session import SharedSessionObject

        eng = self.engine
        t = eng.sessions
        st = eng.store
        s = self._slot(i)
        sid = self.session_id(i)
        sso = SharedSessionObject(SessionConfig(), creator_did=st.did(int(t.sess_creator[s])), session_id=sid)
        sso.state = {0: SessionState.CREATED, 1: SessionState.HANDSHAKING, 2: SessionState.ACTIVE,
                     3: SessionState.TERMINATING, 4: SessionState.ARCHIVED}[int(t.sess_state[s])]
        sso.created_at = _clock.from_us(int(t.sess_created_us[s]))
        te = int(t.sess_terminated_us[s])
        sso.terminated_at = _clock.from_us(te) if te else None
        did = None
        for p in range(int(t.part_count[s])):
            did = st.did(int(t.part_agent[s, p]))
            sso._participants[did] = SessionParticipant(
                agent_did=did,
                ring=ExecutionRing(int(t.part_ring[s, p])),
                sigma_raw=float(t.part_sigma_raw[s, p]),
                sigma_eff=float(t.part_sigma_eff[s, p]),
                joined_at=_clock.from_us(int(t.part_joined_us[s, p])),
            )
        m = ManagedSession(sso)
        parent = None
        for d in range(int(t.delta_count[s])):
            changes = [
                VFSChange(path=p.format(i=d), operation=o.format(i=d),
                          content_hash=h.format(i=d) if h is not None else None)
                for (p, o, h) in self.change_specs
            ]
            sd = SemanticDelta(
                delta_id=f"delta:{d + 1}", turn_id=d + 1, session_id=sid, agent_did=did or "",
                timestamp=_clock.from_us(self.now_us + d + 1), changes=changes, parent_hash=parent,
                delta_hash=self.delta_hash_hex(i, d),
            )
            m.delta_engine._deltas.append(sd)
            m.delta_engine._turn_counter += 1
            parent = sd.delta_hash
        return m


class GovernanceEngine:
    def __init__(
        self,
        device: Optional[str] = None,
        session_capacity: Optional[int] = None,
        agent_capacity: Optional[int] = None,
        dmax: int = 8,
        seed: Optional[int] = None,
        creator_did: str = "did:mesh:admin",
        participant_rows: int = 16,
    ) -> None:
        self.device = resolve_device(device)
        cap = int(session_capacity or min(RUNTIME.session_capacity, 1 << 20))
        if not 1 <= dmax <= 8:
            raise ValueError("dmax must be in [1, 8]")
        self.dmax = dmax
        caps = {"S": cap, "G": cap, "T": cap, "D": cap * dmax, "P": participant_rows, "E": 64, "V": 64,
                "X": 1 << 16, "B": 64}
        self.store = GovernanceStore(str(self.device), caps=caps, max_caps={k: caps[k] for k in "SGTDEV"})
        self.interner = self.store.pool
        self._status = torch.zeros(cap, dtype=torch.int32, device=self.device)
        self.sessions = EngineSessions(self.store, cap, dmax, self._status)
        self.agents = AgentRegistry(self.store, agent_capacity or min(RUNTIME.agent_capacity, 1 << 20))
        self.gc_retention_us = 90 * 86_400 * 1_000_000  # RetentionPolicy.delta_retention_days
        self.seed = int(seed if seed is not None else int.from_bytes(os.urandom(8), "little") >> 1)
        self.creator_id = self.store.agent_id(creator_did)
        self._next_slot = 0
        self._id_counter = 0
        self._last_specs = None
        self._change_cache: dict = {}
        self._rec_bytes = 0  # arena bytes per delta row of the ring (reserved on first use)
        self._off_base = 0
        self._spread = SpreadCounters(6, self.device)
        self._batches: list[PipelineBatch] = []  # host-cursor batches, newest last (for lookup)
        self.sessions_run = 0

    # -- lookup ------------------------------------------------------------------
    def lookup(self, session_id: str) -> Optional[tuple[PipelineBatch, int]]:
        """(batch, index) of a pipeline session by its id, or None.

        One device compare over the resident ``s_uuid`` column; the slot is then
        attributed to the newest batch that wrote it (the rows are a ring, so an
        evicted session is no longer found)."""
        if not session_id.startswith("session:"):
            return None
        h = session_id[len("session:"):].replace("-", "")
        if len(h) != 32:
            return None
        try:
            words = [int(h[8 * k: 8 * k + 8], 16) for k in range(4)]
        except ValueError:
            return None
        w = torch.tensor(words, dtype=torch.int64).to(torch.int32).to(self.device)
        hit = torch.nonzero((self.sessions.sess_uuid == w).all(dim=1)).flatten()
        if hit.numel() == 0:
            return None
        slot = int(hit[0])
        cap = self.sessions.capacity
        for b in reversed(self._batches):
            i = (slot - b.slot_base) % cap
            if i < b.n:
                return b, i
        return None

    # -- agents ----------------------------------------------------------------
    def register_agents(self, dids: Sequence[str], sigmas) -> torch.Tensor:
        return self.agents.add(dids, sigmas)

    def register_synthetic_agents(self, n: int, seed: int = 0, prefix: str = "did:mesh:agent-") -> torch.Tensor:
        """``n`` agents with random-init σ ~ U[0, 1) (the BASELINE synthetic config)."""
        g = torch.Generator().manual_seed(seed)
        sig = torch.rand(n, generator=g, dtype=torch.float64)
        base = self.agents.count
        return self.register_agents([f"{prefix}{base + k}" for k in range(n)], sig)

    # -- pipeline ----------------------------------------------------------------
    def _changes(self, deltas: int, specs) -> tuple[torch.Tensor, list]:
        key = (deltas, tuple(specs))
        hit = self._change_cache.get(key)
        if hit is not None:
            return hit
        pool = self.store.pool
        rows = []
        for d in range(deltas):
            for p, o, h in specs:
                rows.append([pool.intern(p.format(i=d)), pool.intern(o.format(i=d)),
                             pool.intern(h.format(i=d)) if h is not None else -1, -1])
        t = torch.tensor(rows or [[0, 0, 0, 0]], dtype=torch.int32, device=self.device)
        # each delta's changes fragment is the same for every session of the batch:
        # rendered once here (the device emitter's own code) and copied by the kernel
        # (store_template.h, TemplateArgs::frag), as TemplatePipeline does
        frag = None
        if deltas and os.environ.get("AHV_TEMPLATE_FRAG", "1") != "0":
            nch = len(specs)
            words, offs, lens = [], [], []
            for d in range(deltas):
                b = C.render_fragment(pool._pool, rows[d * nch:(d + 1) * nch], d + 1, d > 0)
                offs.append(sum(len(x) for x in words))
                lens.append(len(b))
                words.append(np.frombuffer(b + b"\0" * (-len(b) % 4), dtype=">u4").astype(np.uint32))
            dev = self.device
            frag = (torch.from_numpy(np.concatenate(words).view(np.int32).copy()).to(dev),
                    torch.tensor(offs, dtype=torch.int32, device=dev), torch.tensor(lens, dtype=torch.int32,
                                                                                    device=dev))
        self._change_cache[key] = (t, rows, frag)
        return t, rows, frag

    def _ensure_arena(self, rows: list, deltas: int, nch: int) -> int:
        """Reserve the ring's arena (one record slot per delta row) large enough for
        the longest record this batch can produce; returns that record's padded size."""
        need = max((_record_cap(self.store, rows[d * nch:(d + 1) * nch], d + 1, self.agents.max_did)
                    for d in range(deltas)), default=64)
        if need <= self._rec_bytes:
            return need
        st = self.store
        rec = (need + need // 4 + 63) & ~63
        cap, dmax = self.sessions.capacity, self.dmax
        # a fresh contiguous region past everything reserved so far (the ring's delta
        # rows are addressed by row·rec from its base; the store's delta allocator is
        # not involved: the engine owns every row of its store)
        off = (self._off_base + cap * dmax * self._rec_bytes + 63) & ~63
        self.synchronize()
        st._c.grow_payload(off + cap * dmax * rec)
        st.caps["B"] = st._c.payload_cap
        self._off_base, self._rec_bytes = off, rec
        return need

    def run_pipeline(
        self,
        n: int,
        agents: Optional[torch.Tensor] = None,
        deltas: int = 3,
        changes: Optional[list] = None,
        now_us: Optional[int] = None,
        audit: bool = True,
        max_participants: int = 10,
        min_sigma_eff: float = 0.60,
        stats: Optional[torch.Tensor] = None,
        cursor: Optional[torch.Tensor] = None,
        events=None,
        fold: bool = True,
    ) -> PipelineBatch:
        """Run the full governance pipeline for ``n`` new sessions (asynchronously
        on the current stream).

        ``stats`` (int64[6], on the engine device) accumulates the batch counters
        sessions / ok / participants / deltas / commitments / archived.

        ``events`` (:class:`agent_hypervisor_amd.runtime.events.DeviceEventRing`)
        collects the lifecycle events of every session on the device (N08).

        ``cursor`` (int64[3] on the engine device: slot_base, id_base, now_us)
        makes the launch read its bases from device memory instead of the host
        counters — the graph-capturable form used by
        :class:`agent_hypervisor_amd.runtime.graphs.PipelineGraph`, which also
        advances the cursor on the device.  The host counters are not touched.

        ``fold=False``: leave the batch counters in the engine's spread rows
        (``_spread``); the caller folds them (the graph's fused epilogue does).
        """
        if stats is not None and (stats.dtype != torch.int64 or stats.numel() != 6 or stats.device != self.device):
            raise ValueError("stats must be an int64[6] tensor on the engine device")
        cap = self.sessions.capacity
        if n > cap:
            raise ValueError(f"batch of {n} exceeds session capacity {cap}")
        if self.agents.count == 0:
            raise RuntimeError("register agents before running the pipeline")
        if not 0 <= deltas <= self.dmax:
            raise ValueError(f"deltas must be in [0, {self.dmax}]")
        if agents is None:
            agents = torch.arange(n, dtype=torch.int32, device=self.device) % self.agents.count
        agents = agents.to(self.device, torch.int32).contiguous()
        if agents.numel() != n:
            raise ValueError("agents must have one entry per session")
        specs = changes or REFERENCE_CHANGES
        if len(specs) > 4:
            raise ValueError("at most 4 changes per delta")
        self._last_specs = list(specs)
        ch, rows, frag = self._changes(deltas, specs)
        need = self._ensure_arena(rows, deltas, len(specs))
        st = self.store
        pb, po, pl = st.pool.device_view(self.device)
        now = int(now_us if now_us is not None else _clock.now_us())
        slot_base, id_base = self._next_slot, self._id_counter
        args = {
            "n": n, "slot": 0, "gslot": 0, "tslot": 0, "drow": 0, "doff": 0,
            "session_agent": agents.data_ptr(), "agent_id": self.agents.store_id.data_ptr(),
            "agent_pool": self.agents.did.data_ptr(), "agent_sigma": self.agents.sigma.data_ptr(),
            "changes": ch.data_ptr(), "pool_bytes": pb.data_ptr(), "pool_off": po.data_ptr(),
            "pool_len": pl.data_ptr(), "deltas": deltas, "nch": len(specs), "creator": self.creator_id,
            "maxpart": int(max_participants), "minsig": float(min_sigma_eff), "audit": int(bool(audit)),
            "t0": now, "seed": self.seed, "id_base": id_base, "gc_retention_us": int(self.gc_retention_us),
            "status": self._status.data_ptr() if cursor is None else None,
            "stats": self._spread.begin().data_ptr() if stats is not None else None,
            "ring_cap": cap, "slot_base": slot_base, "dstride": self.dmax, "rec_bytes": self._rec_bytes,
            "off_base": self._off_base, "id_stride": 3,
            "cursor": cursor.data_ptr() if cursor is not None else None,
            "max_rec": need,  # the longest record (the ring slot is larger): small-batch kernel choice
        }
        if frag is not None:
            args.update(frag=frag[0].data_ptr(), frag_off=frag[1].data_ptr(), frag_len=frag[2].data_ptr())
        if cursor is not None:
            if cursor.dtype != torch.int64 or cursor.numel() not in (3, 4) or cursor.device != self.device:
                raise ValueError("cursor must be an int64[3] (or [4]) tensor on the engine device")
        if events is not None:  # DeviceEventRing (N08): lifecycle records appended by the kernel
            ev_scalars, ev_tensors = events.kernel_args()
            args.update(ev_scalars)
            args.update({k: v.data_ptr() for k, v in ev_tensors.items()})
        _pipeline_op.run(st, args, {"merkle_root": self.sessions.merkle_root, "delta_hash": self.sessions.delta_hash,
                                    "status": self._status})
        if stats is not None and fold:
            self._spread.add_into(stats)
        self._keep = (agents, ch, frag)
        if cursor is not None:
            return PipelineBatch(self, -1, n, -1, -1, deltas, list(specs), agents)
        self._next_slot = (slot_base + n) % cap
        self._id_counter = id_base + 3 * n
        self.sessions_run += n
        batch = PipelineBatch(self, slot_base, n, id_base, now, deltas, list(specs), agents)
        # keep only the batches whose rows can still be live (the rows are a ring)
        live, covered = [], n
        for b in reversed(self._batches):
            if covered >= cap:  # every row of b (and of anything older) was overwritten
                break
            live.append(b)
            covered += b.n
        self._batches = live[::-1] + [batch]
        return batch

    def synchronize(self) -> None:
        if self.device.type == "cuda":
            torch.cuda.synchronize(self.device)


def timed(fn, *a, **k):
    t0 = time.perf_counter()
    r = fn(*a, **k)
    return r, time.perf_counter() - t0
