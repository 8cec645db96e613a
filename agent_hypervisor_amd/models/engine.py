"""GovernanceEngine: the batched, device-resident governance pipeline.

This is the MI355X data plane behind :class:`hypervisor.Hypervisor`.  Where the
scalar API runs one session operation at a time on the host, the engine runs the
reference benchmark's full governance pipeline (bench_hypervisor.py:217-239) for
a whole batch of sessions in one gfx950 launch:

    create → join (σ ring gate) → activate → D × audit capture (canonical JSON +
    SHA-256 Merkle chain) → saga create/add/execute → terminate (Merkle root,
    commitment, bond release, GC, archive)

with all state in :mod:`agent_hypervisor_amd.models.tables` SoA tensors.  Ids
(session / saga / step uuid4) are minted on device from a counter-based
generator, timestamps come from one injected ``now_us`` per batch (N09), and
every digest is byte-identical to what the scalar path computes for the same
ids and timestamps (``tests/test_engine_host.py``, ``tests/test_gpu_pipeline.py``).

Multi-GPU: one engine per rank; sessions are sharded by rank (P01), see
:mod:`agent_hypervisor_amd.parallel.directory`.  Steady-state batches can be
captured in a hipGraph with :class:`agent_hypervisor_amd.runtime.graphs.PipelineGraph`.
"""

from __future__ import annotations

import os
import time
from dataclasses import dataclass
from typing import Optional, Sequence

import torch

from agent_hypervisor_amd._native import C  # noqa: F401 - loads the native extension (fails loudly when missing)
from agent_hypervisor_amd.models.tables import AgentTable, SessionTable, VouchSlab
from agent_hypervisor_amd.ops import pipeline as _pipeline_op
from agent_hypervisor_amd.utils.interner import Interner
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
        return "saga:" + _uuid_str(self.engine.sessions.saga_uuid[self._slot(i)].cpu())

    def step_id(self, i: int) -> str:
        return "step:" + _uuid_str(self.engine.sessions.step_uuid[self._slot(i)].cpu())

    def merkle_root_hex(self, i: int) -> str:
        return _u32_hex(self.engine.sessions.merkle_root[self._slot(i)].cpu())

    def delta_hash_hex(self, i: int, d: int) -> str:
        return _u32_hex(self.engine.sessions.delta_hash[self._slot(i), d].cpu())

    def roots(self) -> torch.Tensor:
        return self.engine.sessions.merkle_root.index_select(0, self.slots())

    def status(self) -> torch.Tensor:
        return self.engine.sessions.status.index_select(0, self.slots())

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
        s = self._slot(i)
        sid = self.session_id(i)
        sso = SharedSessionObject(SessionConfig(), creator_did=eng.interner.str(eng.creator_id), session_id=sid)
        sso.state = {0: SessionState.CREATED, 1: SessionState.HANDSHAKING, 2: SessionState.ACTIVE,
                     3: SessionState.TERMINATING, 4: SessionState.ARCHIVED}[int(t.sess_state[s])]
        sso.created_at = _clock.from_us(int(t.sess_created_us[s]))
        te = int(t.sess_terminated_us[s])
        sso.terminated_at = _clock.from_us(te) if te else None
        did = None
        for p in range(int(t.part_count[s])):
            a = int(t.part_agent[s, p])
            did = eng.interner.str(int(eng.agents.did[a]))
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
        vouch_stride: int = 16,
        dmax: int = 8,
        seed: Optional[int] = None,
        creator_did: str = "did:mesh:admin",
    ) -> None:
        self.device = resolve_device(device)
        self.interner = Interner()
        self.sessions = SessionTable(session_capacity or min(RUNTIME.session_capacity, 1 << 20), self.device, dmax)
        self.agents = AgentTable(agent_capacity or min(RUNTIME.agent_capacity, 1 << 20), self.device)
        self.vouches = VouchSlab(self.sessions.capacity, vouch_stride, self.device)
        self.gc_retention_us = 90 * 86_400 * 1_000_000  # RetentionPolicy.delta_retention_days
        self.seed = int(seed if seed is not None else int.from_bytes(os.urandom(8), "little") >> 1)
        self.creator_id = self.interner.intern(creator_did)
        self._next_slot = 0
        self._id_counter = 0
        self._last_specs = None
        self._change_cache: dict = {}
        self._spread = SpreadCounters(6, self.device)
        self._batches: list[PipelineBatch] = []  # host-cursor batches, newest last (for lookup)
        self.sessions_run = 0

    # -- lookup ------------------------------------------------------------------
    def lookup(self, session_id: str) -> Optional[tuple[PipelineBatch, int]]:
        """(batch, index) of a pipeline session by its id, or None.

        One device compare over the resident ``sess_uuid`` column; the slot is
        then attributed to the newest batch that wrote it (the session table is
        a ring, so an overwritten session is no longer found)."""
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
        ids = torch.tensor(self.interner.intern_many(dids), dtype=torch.int32)
        sig = torch.as_tensor(sigmas, dtype=torch.float64)
        return self.agents.add(ids, sig)

    def register_synthetic_agents(self, n: int, seed: int = 0, prefix: str = "did:mesh:agent-") -> torch.Tensor:
        """``n`` agents with random-init σ ~ U[0, 1) (the BASELINE synthetic config)."""
        g = torch.Generator().manual_seed(seed)
        sig = torch.rand(n, generator=g, dtype=torch.float64)
        base = self.agents.count
        return self.register_agents([f"{prefix}{base + k}" for k in range(n)], sig)

    # -- pipeline ----------------------------------------------------------------
    def _changes(self, deltas: int, specs) -> torch.Tensor:
        key = (deltas, tuple(specs))
        hit = self._change_cache.get(key)
        if hit is not None:
            return hit
        rows = []
        for d in range(deltas):
            for p, o, h in specs:
                rows.append([
                    self.interner.intern(p.format(i=d)),
                    self.interner.intern(o.format(i=d)),
                    self.interner.intern(h.format(i=d)) if h is not None else -1,
                    -1,
                ])
        t = torch.tensor(rows, dtype=torch.int32, device=self.device)
        self._change_cache[key] = t
        return t

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
        """
        if stats is not None and (stats.dtype != torch.int64 or stats.numel() != 6 or stats.device != self.device):
            raise ValueError("stats must be an int64[6] tensor on the engine device")
        cap = self.sessions.capacity
        if n > cap:
            raise ValueError(f"batch of {n} exceeds session capacity {cap}")
        if self.agents.count == 0:
            raise RuntimeError("register agents before running the pipeline")
        if agents is None:
            agents = torch.arange(n, dtype=torch.int32, device=self.device) % self.agents.count
        agents = agents.to(self.device, torch.int32).contiguous()
        if agents.numel() != n:
            raise ValueError("agents must have one entry per session")
        specs = changes or REFERENCE_CHANGES
        self._last_specs = list(specs)
        ch = self._changes(deltas, specs)
        pool_b, pool_o, pool_l = self.interner.device_view(self.device)
        now = int(now_us if now_us is not None else _clock.now_us())
        slot_base, id_base = self._next_slot, self._id_counter
        v = self.vouches
        scalars = dict(
            vouch_stride=v.stride, gc_retention_us=int(self.gc_retention_us),
            n=n, slot_base=slot_base, capacity=cap, deltas=deltas, nch=len(specs), dmax=self.sessions.dmax,
            max_participants=max_participants, min_sigma_eff=float(min_sigma_eff), now_us=now,
            seed=self.seed, id_base=id_base, creator_id=self.creator_id, audit=int(bool(audit)),
        )
        tensors = dict(
            session_agent=agents, agent_sigma=self.agents.sigma, agent_did=self.agents.did, changes=ch,
            vouch_count=v.count, vouch_active=v.active if v.allocated else None,
            vouch_released_us=v.released_us if v.allocated else None,
            pool_bytes=pool_b, pool_off=pool_o, pool_len=pool_l,
            stats=self._spread.begin() if stats is not None else None,
        )
        tensors.update({k: getattr(self.sessions, k) for k in SessionTable.COLUMNS})
        if events is not None:  # DeviceEventRing (N08): lifecycle records appended by the kernel
            ev_scalars, ev_tensors = events.kernel_args()
            scalars.update(ev_scalars)
            tensors.update(ev_tensors)
        if cursor is not None:
            if cursor.dtype != torch.int64 or cursor.numel() != 3 or cursor.device != self.device:
                raise ValueError("cursor must be an int64[3] tensor on the engine device")
            tensors["cursor"] = cursor
            _pipeline_op.run(scalars, tensors)
            if stats is not None:
                self._spread.add_into(stats)
            return PipelineBatch(self, -1, n, -1, -1, deltas, list(specs), agents)
        _pipeline_op.run(scalars, tensors)
        if stats is not None:
            self._spread.add_into(stats)
        self._next_slot = (slot_base + n) % cap
        self._id_counter = id_base + 3 * n
        self.sessions_run += n
        batch = PipelineBatch(self, slot_base, n, id_base, now, deltas, list(specs), agents)
        # keep only the batches whose rows can still be live (the table is a ring)
        live, covered = [], n
        for b in reversed(self._batches):
            if covered >= cap:  # every row of b (and of anything older) was overwritten
                break
            live.append(b)
            covered += b.n
        self._batches = live[::-1] + [batch]
        return batch

    def stage_vouches(self, slots, voucher, vouchee, bonded, expiry_us=None) -> torch.Tensor:
        """Record vouch edges of the sessions in ``slots`` (participant-local
        voucher/vouchee indices) in the resident slab; the pipeline's terminate
        stage releases them (K07).  Returns the flat edge indices."""
        return self.vouches.stage(slots, voucher, vouchee, bonded, expiry_us)

    def synchronize(self) -> None:
        if self.device.type == "cuda":
            torch.cuda.synchronize(self.device)


def timed(fn, *a, **k):
    t0 = time.perf_counter()
    r = fn(*a, **k)
    return r, time.perf_counter() - t0
