"""Sharded Hypervisor: one process per GPU, sessions placed by rank (P01).

Every rank runs a local :class:`hypervisor.Hypervisor` over its own device
store (``Hypervisor(device="cuda")`` — the rank's MI355X holds the state of the
sessions it owns).  :class:`ShardedHypervisor` is the SPMD façade over them:
every rank calls the same method in the same order (as in any
``torch.distributed`` program), the :class:`SessionDirectory` — replicated, so
every rank computes the same placement without a round trip — names the owner,
the owner executes, and its result (or exception) is broadcast on the control
group.  Per-session calls therefore touch one GPU; the agent-global views
combine all ranks with the collectives of SURVEY §2.13:

=======================================  ======================================
reference route (api/server.py)          collective
=======================================  ======================================
``GET /api/v1/stats`` (:145-163)         X04 all-reduce of the counters
``GET /agents/{did}/ring`` (:319-331)    X05 all-reduce MIN of (creation seq, ring)
``GET /agents/{did}/liability`` (:570)   X01: (seq, bond) pairs gathered and summed
                                         in global vouch order (bit-exact with one
                                         rank); dense [A] fp64 all-reduce for the
                                         whole population (:meth:`exposure_vector`)
saga lookups by id (:418-505)            X07 routing table (no collective)
Nexus cache invalidation                 X08 broadcast of agent ids
=======================================  ======================================

Control messages (requests, results, exceptions) travel on a CPU ``gloo`` group
(:func:`control_group`); dense device tensors (X01/X04/X05) use the default
group — RCCL over xGMI on MI355X.  :func:`serve_followers` lets ranks ≠ 0 mirror
a driver on rank 0 (the REST front-end of :mod:`hypervisor.api.sharded`).
"""

from __future__ import annotations

import asyncio
from typing import Any, Callable, Optional

import torch
import torch.distributed as dist

from agent_hypervisor_amd.parallel.directory import SessionDirectory, stable_rank
from hypervisor.models import SessionConfig

_CTRL = {}


def control_group():
    """A CPU (gloo) group spanning the default group, for pickled control messages."""
    if not dist.is_initialized():
        return None
    key = dist.get_world_size()
    g = _CTRL.get(key)
    if g is None:
        g = dist.new_group(backend="gloo") if dist.get_backend() != "gloo" else dist.group.WORLD
        _CTRL[key] = g
    return g


def _tensor_device() -> torch.device:
    if dist.is_initialized() and dist.get_backend() == "nccl":
        return torch.device("cuda", torch.cuda.current_device())
    return torch.device("cpu")


class ShardedHypervisor:
    """SPMD façade over per-rank device-backed hypervisors (collective calls)."""

    def __init__(self, device: Optional[str] = None, policy: str = "round_robin", single: bool = False,
                 **hv_kwargs) -> None:
        from hypervisor import Hypervisor

        # single=True: a one-rank façade inside a multi-rank job (reference answers in tests)
        self.rank = 0 if single or not dist.is_initialized() else dist.get_rank()
        self.world = 1 if single or not dist.is_initialized() else dist.get_world_size()
        self.group = None if self.world == 1 else control_group()
        self.local = Hypervisor(device=device, **hv_kwargs)
        self.directory = SessionDirectory(self.world, policy)
        self._session_seq: dict[str, int] = {}  # global creation order (replicated)
        self._vouch_seq = 0
        self._vouch_meta: dict[str, tuple[int, str]] = {}  # vouch id → (global seq, session) on the owner
        self._step_owner: dict[str, str] = {}  # step id → saga id (replicated)
        # live membership: global ranks still serving; after a failover the control and
        # data collectives move to sub-groups of the survivors (global rank ids stay)
        self.members = list(range(self.world))
        self.data_group = None  # default group (RCCL on MI355X) until a failover
        self.heartbeat = None
        self.failovers: list[dict] = []

    # -- control plane ---------------------------------------------------------
    def _bcast(self, obj: Any, src: int) -> Any:
        if self.world == 1:
            return obj
        box = [obj]
        dist.broadcast_object_list(box, src=src, group=self.group)
        return box[0]

    def _gather(self, obj: Any) -> list:
        if self.world == 1:
            return [obj]
        out: list = [None] * len(self.members)
        dist.all_gather_object(out, obj, group=self.group)
        return out

    def _all_reduce(self, t: torch.Tensor, op) -> None:
        if self.world > 1:
            dist.all_reduce(t, op=op, group=self.data_group)

    async def _on(self, owner: int, fn: Callable[[], Any]) -> Any:
        """Run ``fn`` on the owner rank; every rank returns its result or raises its exception."""
        msg = None
        if self.rank == owner:
            try:
                r = fn()
                if asyncio.iscoroutine(r):
                    r = await r
                msg = ("ok", r)
            except Exception as e:  # noqa: BLE001 - re-raised on every rank
                msg = ("err", e)
        msg = self._bcast(msg, owner)
        if msg[0] == "err":
            raise msg[1]
        return msg[1]

    def owner(self, session_id: str) -> int:
        r = self.directory.owner(session_id)
        if r is None:  # liability sessions that are not hypervisor sessions (e.g. "s1")
            r = stable_rank(session_id, self.world)
            if r not in self.members:
                r = self.members[stable_rank(session_id, len(self.members))]
        return r

    def _owner_strict(self, session_id: str) -> int:
        r = self.directory.owner(session_id)
        if r is None:
            raise ValueError(f"Session {session_id} not found")
        return r

    # -- lifecycle (per-session: one GPU) ----------------------------------------
    async def create_session(self, config: SessionConfig, creator_did: str) -> str:
        owner = self.directory.next_rank()

        async def make():
            m = await self.local.create_session(config, creator_did)
            return m.sso.session_id

        sid = await self._on(owner, make)
        self.directory.assign(sid, owner)
        self._session_seq[sid] = len(self._session_seq)
        return sid

    async def join_session(self, session_id: str, agent_did: str, **kw):
        return await self._on(self._owner_strict(session_id),
                              lambda: self.local.join_session(session_id, agent_did, **kw))

    async def activate_session(self, session_id: str) -> None:
        await self._on(self._owner_strict(session_id), lambda: self.local.activate_session(session_id))

    async def terminate_session(self, session_id: str) -> Optional[str]:
        return await self._on(self._owner_strict(session_id), lambda: self.local.terminate_session(session_id))

    async def verify_behavior(self, session_id: str, agent_did: str, claimed, observed, action_id=None):
        return await self._on(self._owner_strict(session_id),
                              lambda: self.local.verify_behavior(session_id, agent_did, claimed, observed, action_id))

    def _summary(self, session_id: str) -> dict:
        m = self.local.get_session(session_id)
        if m is None:
            raise ValueError(f"Session {session_id} not found")
        sso = m.sso
        return {
            "session_id": sso.session_id, "state": sso.state.value, "consistency_mode": sso.consistency_mode.value,
            "creator_did": sso.creator_did, "created_at": sso.created_at.isoformat(), "rank": self.rank,
            "participants": [
                {"agent_did": p.agent_did, "ring": int(p.ring), "sigma_raw": p.sigma_raw, "sigma_eff": p.sigma_eff,
                 "is_active": p.is_active} for p in sso.participants
            ],
            "turn_count": m.delta_engine.turn_count,
            "sagas": [g.saga_id for g in m.saga.sagas],
        }

    async def get_session(self, session_id: str) -> dict:
        return await self._on(self._owner_strict(session_id), lambda: self._summary(session_id))

    async def capture(self, session_id: str, agent_did: str, changes: list, delta_id: Optional[str] = None) -> str:
        def cap():
            m = self.local._get_session(session_id)
            return m.delta_engine.capture(agent_did, changes, delta_id).delta_hash

        return await self._on(self._owner_strict(session_id), cap)

    async def merkle_root(self, session_id: str) -> Optional[str]:
        return await self._on(self._owner_strict(session_id),
                              lambda: self.local._get_session(session_id).delta_engine.compute_merkle_root())

    # -- liability (session-scoped → the owner's device) ---------------------------
    async def vouch(self, voucher_did: str, vouchee_did: str, session_id: str, voucher_sigma: float,
                    bond_pct: Optional[float] = None, expiry=None) -> dict:
        owner = self.owner(session_id)
        seq = self._vouch_seq
        self._vouch_seq += 1

        def do():
            v = self.local.vouching.vouch(voucher_did, vouchee_did, session_id, voucher_sigma, bond_pct, expiry)
            self._vouch_meta[v.vouch_id] = (seq, session_id)
            return _vouch_dict(v)

        return await self._on(owner, do)

    async def compute_sigma_eff(self, vouchee_did: str, session_id: str, sigma: float, risk_weight: float) -> float:
        return await self._on(self.owner(session_id),
                              lambda: self.local.vouching.compute_sigma_eff(vouchee_did, session_id, sigma, risk_weight))

    async def get_total_exposure(self, voucher_did: str, session_id: str) -> float:
        return await self._on(self.owner(session_id),
                              lambda: self.local.vouching.get_total_exposure(voucher_did, session_id))

    async def release_session_bonds(self, session_id: str) -> int:
        return await self._on(self.owner(session_id), lambda: self.local.vouching.release_session_bonds(session_id))

    async def slash(self, vouchee_did: str, session_id: str, vouchee_sigma: float, risk_weight: float, reason: str,
                    agent_scores: dict) -> dict:
        """Owner-executed slash (K06); the caller's score dict is updated on every rank."""

        def do():
            scores = dict(agent_scores)
            res = self.local.slashing.slash(vouchee_did, session_id, vouchee_sigma, risk_weight, reason, scores)
            return {"slash_id": res.slash_id, "scores": scores,
                    "clips": [(c.voucher_did, c.sigma_before, c.sigma_after) for c in res.voucher_clips]}

        out = await self._on(self.owner(session_id), do)
        agent_scores.clear()
        agent_scores.update(out["scores"])
        return out

    # -- sagas (X07 routing) ---------------------------------------------------------
    async def create_saga(self, session_id: str) -> str:
        owner = self._owner_strict(session_id)
        gid = await self._on(owner, lambda: self.local._get_session(session_id).saga.create_saga(session_id).saga_id)
        self.directory.register_saga(gid, session_id)
        return gid

    def _route(self, saga_id: str) -> tuple[int, str]:
        r = self.directory.route_saga(saga_id)
        if r is None:
            from hypervisor.saga.state_machine import SagaStateError

            raise SagaStateError(f"Saga {saga_id} not found")
        return r

    async def add_step(self, saga_id: str, action_id: str, agent_did: str, execute_api: str,
                       undo_api: Optional[str] = None, timeout_seconds: int = 300, max_retries: int = 0) -> str:
        owner, sid = self._route(saga_id)
        step_id = await self._on(owner, lambda: self.local._get_session(sid).saga.add_step(
            saga_id, action_id, agent_did, execute_api, undo_api, timeout_seconds, max_retries).step_id)
        self._step_owner[step_id] = saga_id
        return step_id

    async def execute_step(self, saga_id: str, step_id: str, executor: Callable[..., Any]) -> Any:
        owner, sid = self._route(saga_id)
        return await self._on(owner, lambda: self.local._get_session(sid).saga.execute_step(saga_id, step_id, executor))

    async def compensate(self, saga_id: str, compensator: Callable[..., Any]) -> list[str]:
        owner, sid = self._route(saga_id)

        async def do():
            failed = await self.local._get_session(sid).saga.compensate(saga_id, compensator)
            return [s.step_id for s in failed]

        return await self._on(owner, do)

    async def get_saga(self, saga_id: str) -> dict:
        owner, sid = self._route(saga_id)
        return await self._on(owner, lambda: self.local._get_session(sid).saga.get_saga(saga_id).to_dict())

    # -- agent-global views (collectives) -------------------------------------------------
    def stats(self) -> dict:
        """X04: session / participant / saga / vouch totals summed over ranks."""
        hv = self.local
        snaps = hv.snapshots()  # one batched device read
        sagas = hv.saga_summaries()
        vals = [
            len(snaps), sum(1 for x in snaps if x.state.value not in ("archived", "terminating")),
            sum(x.participant_count for x in snaps),
            sum(1 for g in sagas if g["state"] in ("running", "compensating")), len(hv.vouching.records()),
            len(sagas),
        ]
        t = torch.tensor(vals, dtype=torch.int64, device=_tensor_device() if self.world > 1 else "cpu")
        self._all_reduce(t, dist.ReduceOp.SUM)
        keys = ("total_sessions", "active_sessions", "total_participants", "active_sagas", "total_vouches",
                "total_sagas")
        return dict(zip(keys, (int(x) for x in t.tolist())))

    def agent_ring(self, agent_did: str) -> Optional[dict]:
        """X05: the agent's ring in the earliest-created session where it is an
        active participant (reference: first match in ``_sessions`` order)."""
        big = 1 << 62
        best, best_sid, best_ring = big, None, None
        for x in self.local.snapshots(parts=True):  # local creation order, one batched read
            sid = x.session_id
            for p in x.participants:
                if p.agent_did == agent_did and p.is_active:
                    key = (self._session_seq[sid] << 8) | int(p.ring)
                    if key < best:
                        best, best_sid, best_ring = key, sid, int(p.ring)
                    break
        t = torch.tensor([best], dtype=torch.int64, device=_tensor_device() if self.world > 1 else "cpu")
        self._all_reduce(t, dist.ReduceOp.MIN)
        key = int(t.item())
        if key >= big:
            return None
        seq = key >> 8
        sid = next(s for s, q in self._session_seq.items() if q == seq)
        return {"agent_did": agent_did, "ring": key & 0xFF, "session_id": sid}

    def agent_liability(self, agent_did: str) -> dict:
        """X01 for one agent: vouches given/received across all ranks in global
        vouch order; exposure = Σ live bonds given, summed in that order."""
        mine = []
        for v in self.local.vouching.records():
            if v.voucher_did == agent_did or v.vouchee_did == agent_did:
                seq = self._vouch_meta.get(v.vouch_id, (1 << 62, ""))[0]
                mine.append((seq, _vouch_dict(v)))
        allv = sorted((x for part in self._gather(mine) for x in part), key=lambda x: x[0])
        given = [d for _, d in allv if d["voucher_did"] == agent_did]
        received = [d for _, d in allv if d["vouchee_did"] == agent_did]
        exposure = 0.0
        for d in given:
            if d["is_active"] and not d["is_expired"]:
                exposure += d["bonded_amount"]
        return {"agent_did": agent_did, "vouches_given": given, "vouches_received": received,
                "total_exposure": exposure}

    def exposure_vector(self, agent_ids: dict[str, int], n_agents: int) -> torch.Tensor:
        """X01 dense: per-agent live bonded exposure over every rank's sessions as
        one [A] fp64 all-reduce (RCCL over xGMI on MI355X)."""
        dev = _tensor_device()
        x = torch.zeros(n_agents, dtype=torch.float64)
        for v in self.local.vouching.records():
            k = agent_ids.get(v.voucher_did)
            if k is not None and v.is_live:
                x[k] += v.bonded_amount
        x = x.to(dev)
        self._all_reduce(x, dist.ReduceOp.SUM)
        return x

    def list_sessions(self, state: Optional[str] = None) -> list[dict]:
        local = []
        for x in self.local.snapshots():
            sid = x.session_id
            st = x.state.value
            if state is None or st == state:
                local.append((self._session_seq.get(sid, 1 << 62),
                              {"session_id": sid, "state": st, "participant_count": x.participant_count,
                               "rank": self.rank}))
        return [d for _, d in sorted((x for part in self._gather(local) for x in part), key=lambda x: x[0])]

    # -- resilience: heartbeat, checkpoint, failover -----------------------
    def start_heartbeat(self, interval_s: float = 0.5):
        """Stamp this rank's liveness in the rendezvous store every ``interval_s``."""
        from agent_hypervisor_amd.parallel.resilience import Heartbeat

        if self.world > 1 and self.heartbeat is None:
            self.heartbeat = Heartbeat(interval_s).start()
        return self.heartbeat

    def dead_ranks(self, timeout_s: float) -> list[int]:
        """Members whose heartbeat is older than ``timeout_s`` (local, no collective)."""
        if self.heartbeat is None:
            return []
        return [r for r in self.heartbeat.dead_ranks(timeout_s) if r in self.members]

    def agree_failed(self, suspects: list[int]) -> list[int]:
        """One failure verdict for all survivors: the lowest member not suspected
        publishes its suspect list in the rendezvous store under the next failover
        epoch and every survivor adopts it (local heartbeat views can differ by a
        beat)."""
        import json

        from agent_hypervisor_amd.parallel.resilience import _store

        st = _store()
        key = f"ahv/failover/{len(self.failovers)}"
        coord = min(r for r in self.members if r not in suspects)
        if self.rank == coord:
            st.set(key, json.dumps(sorted(suspects)))
        st.wait([key])
        return json.loads(st.get(key).decode())

    def checkpoint(self, root: str) -> str:
        """Each rank persists its own sessions (and its share of the vouch
        ordering) under ``root/rank<r>``; collective over the members."""
        import json
        import os

        from agent_hypervisor_amd.runtime.checkpoint import save_hypervisor

        d = save_hypervisor(self.local, os.path.join(root, f"rank{self.rank}"))
        with open(os.path.join(d, "sharded.json"), "w") as f:
            json.dump({"rank": self.rank, "vouch_meta": self._vouch_meta}, f)
        if self.world > 1:
            dist.barrier(group=self.group)
        return d

    async def failover(self, failed: list[int], root: str) -> list[tuple[str, int, int]]:
        """Survivors (every remaining member calls this) re-home the failed
        ranks' sessions (least-loaded first), re-hydrate the ones assigned here
        from the failed ranks' checkpoints — audit chains re-verified on load — and
        move the control/data collectives to sub-groups of the survivors."""
        import json
        import os

        from agent_hypervisor_amd.parallel.resilience import apply_failover, failover_plan, rehydrate

        failed = sorted(set(failed) & set(self.members))
        if not failed:
            return []
        if self.rank in failed:
            raise RuntimeError("a failed rank cannot take part in its own failover")
        moves = failover_plan(self.directory, failed)
        apply_failover(self.directory, moves, failed)
        for f in failed:
            src = os.path.join(root, f"rank{f}")
            mine = [(s, a, b) for s, a, b in moves if a == f and b == self.rank]
            if mine:
                rehydrate(src, mine, self.rank, hv=self.local)
            meta = os.path.join(src, "sharded.json")
            if os.path.exists(meta):
                with open(meta) as fh:
                    vm = json.load(fh)["vouch_meta"]
                moved = {s for s, _, b in mine}
                self._vouch_meta.update({k: tuple(v) for k, v in vm.items() if v[1] in moved})
        self.members = [r for r in self.members if r not in failed]
        # only the survivors synchronise on these groups (the failed ranks never call in)
        self.group = dist.new_group(ranks=self.members, backend="gloo", use_local_synchronization=True)
        self.data_group = dist.new_group(ranks=self.members, use_local_synchronization=True)
        self.failovers.append({"failed": failed, "moves": len(moves)})
        return moves

    def invalidate_agents(self, agent_dids: list[str]) -> list[str]:
        """X08: broadcast Nexus cache invalidations from rank 0 to every rank."""
        dids = self._bcast(list(agent_dids), 0)
        nexus = self.local.nexus
        if nexus is not None:
            for d in dids:
                nexus.invalidate_cache(d)
        return dids


def _vouch_dict(v) -> dict:
    return {
        "vouch_id": v.vouch_id, "voucher_did": v.voucher_did, "vouchee_did": v.vouchee_did,
        "session_id": v.session_id, "bonded_sigma_pct": v.bonded_sigma_pct, "bonded_amount": v.bonded_amount,
        "is_active": bool(v.is_active), "is_expired": bool(v.is_expired),
    }


# ------------------------------------------------------------------ driver / followers

_STOP = "__stop__"


class Driver:
    """Rank 0's handle: each call is broadcast so every rank runs the same
    collective method (followers run :func:`serve_followers`)."""

    def __init__(self, shv: ShardedHypervisor) -> None:
        if shv.rank != 0:
            raise RuntimeError("the driver runs on rank 0")
        self.shv = shv

    async def call(self, name: str, *args, **kwargs):
        self.shv._bcast((name, args, kwargs), 0)
        return await _invoke(self.shv, name, args, kwargs)

    def stop(self) -> None:
        self.shv._bcast(_STOP, 0)


async def _invoke(shv: ShardedHypervisor, name: str, args, kwargs):
    r = getattr(shv, name)(*args, **kwargs)
    if asyncio.iscoroutine(r):
        r = await r
    return r


async def serve_followers(shv: ShardedHypervisor) -> int:
    """Mirror the driver on ranks ≠ 0 until it stops; returns calls served."""
    n = 0
    while True:
        msg = shv._bcast(None, 0)
        if msg == _STOP:
            return n
        name, args, kwargs = msg
        try:
            await _invoke(shv, name, args, kwargs)
        except Exception:  # noqa: BLE001 - the driver raises it; followers keep serving
            pass
        n += 1
