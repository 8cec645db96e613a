"""Sharded Hypervisor: one process per GPU, rank-local serving.

Every rank runs a local :class:`hypervisor.Hypervisor` over its own device store
(``Hypervisor(device="cuda")`` — the rank's MI355X holds the state of the
sessions it owns) and serves requests *independently*:

* **Placement without a directory.**  A session's owner is a stable hash of its
  id over the live ranks (:meth:`ShardedHypervisor.owner`).  A rank creating a
  session mints an id (``session:{uuid4}``) that hashes to the chosen owner —
  itself by default — so every rank routes any session id, liability-session id
  or saga id without a lookup table or a broadcast.
* **Per-session calls** (create/join/activate/capture/terminate, vouch/σ_eff/
  exposure/slash, saga create/add/execute/compensate) run on the owner.  Called
  on the owner they touch no other rank (zero collectives, zero messages —
  :attr:`counters`); called elsewhere they are forwarded point-to-point to the
  owner over the node-local RPC of :mod:`agent_hypervisor_amd.parallel.rpc`
  while every other rank keeps serving.  Executors and compensators cross ranks
  by *name* (:meth:`register_executor` on every rank); local calls take callables.
* **Agent-global views** combine all ranks.  They are sequenced by rank 0 (any
  rank may ask; rank 0 tells every rank to enter the view, so all ranks run the
  view's collectives in the same order):

  =======================================  ======================================
  reference route (api/server.py)          combination
  =======================================  ======================================
  ``GET /api/v1/stats`` (:145-163)         X04 all-reduce of the counters, each
                                           rank's from one batched device read
  ``GET /agents/{did}/ring`` (:319-331)    X05 all-reduce MIN of (creation time,
                                           rank, ring) keys
  ``GET /agents/{did}/liability`` (:570)   the agent's vouch records from every
                                           rank, summed in global vouch order
                                           (bit-exact with one rank)
  dense per-agent exposure                 X01: K04 over each rank's store edge
                                           columns → [A] fp64 all-reduce
  ``GET /api/v1/sessions``                 per-rank snapshots, merged by creation
  =======================================  ======================================

Failure handling: heartbeats, one agreed failure verdict (the first
proposer's list wins), checkpoints per rank, and failover — the dead rank's
sessions *and* liability-only sessions re-home deterministically (to the next
live rank after their home) and are re-hydrated from its checkpoint there.
"""

from __future__ import annotations

import asyncio
import json
import os
from dataclasses import asdict
from datetime import datetime
from typing import Any, Callable, Optional

import torch
import torch.distributed as dist

from agent_hypervisor_amd.parallel.directory import stable_rank
from hypervisor.models import ConsistencyMode, SessionConfig

_CTRL: dict = {}
_EPOCH_US = 1_577_836_800_000_000  # 2020-01-01T00:00:00Z: creation keys are µs after this


def control_group():
    """A CPU (gloo) group spanning the default group (barriers, checkpoints)."""
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


def _cfg_out(c: SessionConfig) -> dict:
    d = asdict(c)
    d["consistency_mode"] = ConsistencyMode(c.consistency_mode).value
    return d


def _cfg_in(d: dict) -> SessionConfig:
    d = dict(d)
    d["consistency_mode"] = ConsistencyMode(d["consistency_mode"])
    return SessionConfig(**d)


def _changes_out(changes) -> list:
    return [{"path": c.path, "operation": c.operation, "content_hash": c.content_hash,
             "previous_hash": c.previous_hash, "agent_did": c.agent_did} for c in changes]


def _changes_in(rows) -> list:
    from hypervisor.audit.delta import VFSChange

    return [VFSChange(path=r["path"], operation=r["operation"], content_hash=r.get("content_hash"),
                      previous_hash=r.get("previous_hash"), agent_did=r.get("agent_did")) for r in rows]


def _us(t: Optional[datetime]) -> int:
    from hypervisor._clock import to_us

    return to_us(t) if t is not None else 0


async def _noop():
    return None


async def _noop_comp(step):
    return None


# per-session methods served for other ranks (the RPC whitelist)
_SERVED = (
    "create_session", "join_session", "activate_session", "terminate_session", "verify_behavior", "get_session",
    "capture", "merkle_root", "vouch", "compute_sigma_eff", "get_total_exposure", "release_session_bonds",
    "slash", "create_saga", "add_step", "execute_step", "compensate", "get_saga",
    "_view", "_view_enter", "_stop",
)


class ShardedHypervisor:
    """Rank-local serving façade over per-rank (device-backed) hypervisors."""

    def __init__(self, device: Optional[str] = None, policy: str = "local", single: bool = False,
                 **hv_kwargs) -> None:
        from hypervisor import Hypervisor

        if policy not in ("local", "round_robin"):
            raise ValueError("policy must be 'local' (create on the calling rank) or 'round_robin'")
        # single=True: a one-rank façade inside a multi-rank job (reference answers in tests)
        self.rank = 0 if single or not dist.is_initialized() else dist.get_rank()
        self.world = 1 if single or not dist.is_initialized() else dist.get_world_size()
        self.policy = policy
        self.local = Hypervisor(device=device, **hv_kwargs)
        self.members = list(range(self.world))
        self._live = frozenset(self.members)
        self.group = None if self.world == 1 else control_group()
        self.data_group = None  # default group (RCCL on MI355X) until a failover
        self.rpc = None
        self.executors: dict[str, Callable[..., Any]] = {"noop": _noop}
        self.compensators: dict[str, Callable[..., Any]] = {"noop": _noop_comp}
        self.counters = {"local": 0, "forwarded": 0, "collectives": 0, "views": 0}
        self._rr = 0
        self._sagas: dict[str, str] = {}  # saga id → session id (sagas this rank owns)
        self._vouch_seq = 0
        self._vouch_key: dict[str, tuple] = {}  # vouch id → global order key (created µs, rank, seq)
        self._view_lock: Optional[asyncio.Lock] = None
        self._stopped: Optional[asyncio.Event] = None
        self.heartbeat = None
        self.failovers: list[dict] = []

    # -- startup / shutdown --------------------------------------------------------
    async def start(self) -> "ShardedHypervisor":
        """Open this rank's RPC endpoint and learn every peer's (all ranks call this)."""
        from agent_hypervisor_amd.parallel.rpc import RpcEndpoint

        self._stopped = asyncio.Event()
        self._view_lock = asyncio.Lock()
        if self.world == 1:
            return self
        from agent_hypervisor_amd.parallel.resilience import _store

        self.rpc = RpcEndpoint(self.rank, self._handle, _SERVED)
        addr = await self.rpc.start()
        st = _store()
        st.set(f"ahv/rpc/{self.rank}", addr)
        loop = asyncio.get_running_loop()
        for r in self.members:
            if r != self.rank:
                self.rpc.peers[r] = (await loop.run_in_executor(None, st.get, f"ahv/rpc/{r}")).decode()
        return self

    async def serve_forever(self) -> None:
        """Keep serving forwarded calls and views until :meth:`shutdown` on rank 0."""
        await self._stopped.wait()

    async def shutdown(self) -> None:
        """Rank 0: stop every rank's :meth:`serve_forever`, then this rank's."""
        if self.rpc is not None and self.rank == self.members[0]:
            await asyncio.gather(*[self.rpc.call(r, "_stop") for r in self.members if r != self.rank],
                                 return_exceptions=True)
        self._stopped.set()

    async def close(self) -> None:
        if self.rpc is not None:
            await self.rpc.close()
            self.rpc = None

    async def _handle(self, name: str, args: list, kwargs: dict) -> Any:
        if name == "_stop":
            self._stopped.set()
            return True
        if name == "_view":
            return await self._view(*args)
        if name == "_view_enter":
            return self._collective(*args)
        return await getattr(self, "_local_" + name)(*args, **kwargs)

    # -- placement ---------------------------------------------------------------------
    def owner(self, key: str) -> int:
        """Owner rank of a session / liability-session / saga id: its home — a stable
        hash over the world — or, when the home rank has failed, the next live rank
        after it.  Re-homing by home rank (not by key) keeps a saga with its session
        (their ids were minted for the same home) on every survivor's routing."""
        h = stable_rank(key, self.world)
        live = self._live
        while h not in live:
            h = (h + 1) % self.world
        return h

    _MINT_TRIES = 1 << 16  # P(no hit) for one live rank of 8 after this many draws: (7/8)^65536

    def _mint(self, prefix: str, target: int) -> str:
        """A fresh ``prefix{uuid4}`` whose owner is ``target`` (a live rank: an id can
        only hash to a live rank, so a dead or unknown target is refused up front)."""
        from agent_hypervisor_amd._native import C

        if target not in self._live:
            raise ValueError(f"rank {target} is not a live member {sorted(self._live)}")
        for _ in range(self._MINT_TRIES):
            k = C.uuid4(prefix)
            if self.owner(k) == target:
                return k
        raise RuntimeError(f"could not mint an id owned by rank {target}")

    async def _route(self, key: str, name: str, *args, **kwargs) -> Any:
        o = self.owner(key)
        if o == self.rank:
            self.counters["local"] += 1
            return await getattr(self, "_local_" + name)(*args, **kwargs)
        self.counters["forwarded"] += 1
        return await self.rpc.call(o, name, *args, **kwargs)

    # -- lifecycle ---------------------------------------------------------------------
    async def create_session(self, config: SessionConfig, creator_did: str, rank: Optional[int] = None) -> str:
        """Create a session on ``rank`` (default: this rank with policy ``local``,
        the next live rank with ``round_robin``); returns its id."""
        if rank is None:
            if self.policy == "local":
                rank = self.rank
            else:
                rank = self.members[self._rr % len(self.members)]
                self._rr += 1
        sid = self._mint("session:", rank)
        return await self._route(sid, "create_session", _cfg_out(config), creator_did, sid)

    async def _local_create_session(self, cfg: dict, creator_did: str, sid: str) -> str:
        m = await self.local.create_session(_cfg_in(cfg), creator_did, session_id=sid)
        return m.sso.session_id

    async def join_session(self, session_id: str, agent_did: str, sigma_raw: float = 0.0, **kw):
        from hypervisor.models import ExecutionRing

        if kw.get("actions"):
            acts = []
            for a in kw["actions"]:
                d = dict(a) if isinstance(a, dict) else asdict(a)
                d["reversibility"] = getattr(d["reversibility"], "value", d["reversibility"])
                acts.append(d)
            kw["actions"] = acts
        return ExecutionRing(await self._route(session_id, "join_session", session_id, agent_did, sigma_raw, **kw))

    async def _local_join_session(self, session_id: str, agent_did: str, sigma_raw: float = 0.0, **kw) -> int:
        if kw.get("actions"):
            from hypervisor.models import ActionDescriptor, ReversibilityLevel

            kw["actions"] = [ActionDescriptor(**dict(a, reversibility=ReversibilityLevel(a["reversibility"])))
                             for a in kw["actions"]]
        return int(await self.local.join_session(session_id, agent_did, sigma_raw=sigma_raw, **kw))

    async def activate_session(self, session_id: str) -> None:
        await self._route(session_id, "activate_session", session_id)

    async def _local_activate_session(self, session_id: str) -> None:
        await self.local.activate_session(session_id)

    async def terminate_session(self, session_id: str) -> Optional[str]:
        return await self._route(session_id, "terminate_session", session_id)

    async def _local_terminate_session(self, session_id: str) -> Optional[str]:
        return await self.local.terminate_session(session_id)

    async def verify_behavior(self, session_id: str, agent_did: str, claimed, observed, action_id=None):
        return await self._route(session_id, "verify_behavior", session_id, agent_did, claimed, observed, action_id)

    async def _local_verify_behavior(self, session_id, agent_did, claimed, observed, action_id=None):
        r = await self.local.verify_behavior(session_id, agent_did, claimed, observed, action_id)
        return None if r is None else {"drift_score": r.drift_score, "severity": r.severity.value,
                                       "passed": r.passed, "should_slash": r.should_slash}

    async def get_session(self, session_id: str) -> dict:
        return await self._route(session_id, "get_session", session_id)

    async def _local_get_session(self, session_id: str) -> dict:
        m = self.local.get_session(session_id)
        if m is None:
            raise ValueError(f"Session {session_id} not found")
        x = self.local.snapshots([m], parts=True)[0]
        return {
            "session_id": x.session_id, "state": x.state.value, "consistency_mode": x.consistency_mode.value,
            "creator_did": x.creator_did, "created_at": x.created_at.isoformat(), "rank": self.rank,
            "participants": [
                {"agent_did": p.agent_did, "ring": int(p.ring), "sigma_raw": p.sigma_raw, "sigma_eff": p.sigma_eff,
                 "is_active": p.is_active} for p in x.participants
            ],
            "turn_count": m.delta_engine.turn_count,
            "sagas": [g.saga_id for g in m.saga.sagas],
        }

    async def capture(self, session_id: str, agent_did: str, changes: list, delta_id: Optional[str] = None) -> str:
        return await self._route(session_id, "capture", session_id, agent_did, _changes_out(changes), delta_id)

    async def _local_capture(self, session_id: str, agent_did: str, changes: list, delta_id=None) -> str:
        m = self.local._get_session(session_id)
        return m.delta_engine.capture(agent_did, _changes_in(changes), delta_id).delta_hash

    async def merkle_root(self, session_id: str) -> Optional[str]:
        return await self._route(session_id, "merkle_root", session_id)

    async def _local_merkle_root(self, session_id: str) -> Optional[str]:
        return self.local._get_session(session_id).delta_engine.compute_merkle_root()

    # -- liability (session-scoped → the owner's device) ---------------------------------
    async def vouch(self, voucher_did: str, vouchee_did: str, session_id: str, voucher_sigma: float,
                    bond_pct: Optional[float] = None, expiry: Optional[datetime] = None) -> dict:
        return await self._route(session_id, "vouch", voucher_did, vouchee_did, session_id, voucher_sigma, bond_pct,
                                 expiry.isoformat() if expiry is not None else None)

    async def _local_vouch(self, voucher_did, vouchee_did, session_id, voucher_sigma, bond_pct=None, expiry=None):
        exp = datetime.fromisoformat(expiry) if expiry else None
        v = self.local.vouching.vouch(voucher_did, vouchee_did, session_id, voucher_sigma, bond_pct, exp)
        self._vouch_seq += 1
        self._vouch_key[v.vouch_id] = (_us(v.created_at), self.rank, self._vouch_seq)
        return _vouch_dict(v)

    async def compute_sigma_eff(self, vouchee_did: str, session_id: str, sigma: float, risk_weight: float) -> float:
        return await self._route(session_id, "compute_sigma_eff", vouchee_did, session_id, sigma, risk_weight)

    async def _local_compute_sigma_eff(self, vouchee_did, session_id, sigma, risk_weight) -> float:
        return self.local.vouching.compute_sigma_eff(vouchee_did, session_id, sigma, risk_weight)

    async def get_total_exposure(self, voucher_did: str, session_id: str) -> float:
        return await self._route(session_id, "get_total_exposure", voucher_did, session_id)

    async def _local_get_total_exposure(self, voucher_did, session_id) -> float:
        return float(self.local.vouching.get_total_exposure(voucher_did, session_id))

    async def release_session_bonds(self, session_id: str) -> int:
        return await self._route(session_id, "release_session_bonds", session_id)

    async def _local_release_session_bonds(self, session_id) -> int:
        return int(self.local.vouching.release_session_bonds(session_id))

    async def slash(self, vouchee_did: str, session_id: str, vouchee_sigma: float, risk_weight: float, reason: str,
                    agent_scores: dict) -> dict:
        """Owner-executed slash (K06); the caller's score dict is updated in place."""
        out = await self._route(session_id, "slash", vouchee_did, session_id, vouchee_sigma, risk_weight, reason,
                                dict(agent_scores))
        agent_scores.clear()
        agent_scores.update(out["scores"])
        out["clips"] = [tuple(c) for c in out["clips"]]
        return out

    async def _local_slash(self, vouchee_did, session_id, vouchee_sigma, risk_weight, reason, scores) -> dict:
        res = self.local.slashing.slash(vouchee_did, session_id, vouchee_sigma, risk_weight, reason, scores)
        return {"slash_id": res.slash_id, "scores": scores,
                "clips": [[c.voucher_did, c.sigma_before, c.sigma_after] for c in res.voucher_clips]}

    # -- sagas (ids route to their session's owner) ---------------------------------------
    async def create_saga(self, session_id: str) -> str:
        gid = self._mint("saga:", self.owner(session_id))
        return await self._route(session_id, "create_saga", session_id, gid)

    async def _local_create_saga(self, session_id: str, gid: str) -> str:
        self.local._get_session(session_id).saga.create_saga(session_id, saga_id=gid)
        self._sagas[gid] = session_id
        return gid

    def _saga_session(self, saga_id: str) -> str:
        sid = self._sagas.get(saga_id)
        if sid is None:
            from hypervisor.saga.state_machine import SagaStateError

            raise SagaStateError(f"Saga {saga_id} not found")
        return sid

    async def add_step(self, saga_id: str, action_id: str, agent_did: str, execute_api: str,
                       undo_api: Optional[str] = None, timeout_seconds: int = 300, max_retries: int = 0) -> str:
        return await self._route(saga_id, "add_step", saga_id, action_id, agent_did, execute_api, undo_api,
                                 timeout_seconds, max_retries)

    async def _local_add_step(self, saga_id, action_id, agent_did, execute_api, undo_api=None, timeout_seconds=300,
                              max_retries=0) -> str:
        orch = self.local._get_session(self._saga_session(saga_id)).saga
        return orch.add_step(saga_id, action_id, agent_did, execute_api, undo_api, timeout_seconds,
                             max_retries).step_id

    def register_executor(self, name: str, fn: Callable[..., Any]) -> None:
        """Make an executor callable by name from any rank (register on every rank)."""
        self.executors[name] = fn

    def register_compensator(self, name: str, fn: Callable[..., Any]) -> None:
        self.compensators[name] = fn

    async def execute_step(self, saga_id: str, step_id: str, executor: Any = "noop") -> Any:
        """``executor``: a registered name (any rank) or a callable (owner rank only)."""
        if callable(executor):
            if self.owner(saga_id) != self.rank:
                raise TypeError("executors cross ranks by name: register_executor() on every rank")
            self.counters["local"] += 1
            return await self._exec_step(saga_id, step_id, executor)
        return await self._route(saga_id, "execute_step", saga_id, step_id, executor)

    async def _local_execute_step(self, saga_id: str, step_id: str, executor: str = "noop") -> Any:
        fn = self.executors.get(executor)
        if fn is None:
            raise KeyError(f"executor {executor!r} is not registered on rank {self.rank}")
        return await self._exec_step(saga_id, step_id, fn)

    async def _exec_step(self, saga_id, step_id, fn):
        orch = self.local._get_session(self._saga_session(saga_id)).saga
        return await orch.execute_step(saga_id, step_id, executor=fn)

    async def compensate(self, saga_id: str, compensator: Any = "noop") -> list[str]:
        if callable(compensator):
            if self.owner(saga_id) != self.rank:
                raise TypeError("compensators cross ranks by name: register_compensator() on every rank")
            self.counters["local"] += 1
            return await self._comp(saga_id, compensator)
        return await self._route(saga_id, "compensate", saga_id, compensator)

    async def _local_compensate(self, saga_id: str, compensator: str = "noop") -> list[str]:
        fn = self.compensators.get(compensator)
        if fn is None:
            raise KeyError(f"compensator {compensator!r} is not registered on rank {self.rank}")
        return await self._comp(saga_id, fn)

    async def _comp(self, saga_id, fn) -> list[str]:
        orch = self.local._get_session(self._saga_session(saga_id)).saga
        return [s.step_id for s in await orch.compensate(saga_id, fn)]

    async def get_saga(self, saga_id: str) -> dict:
        return await self._route(saga_id, "get_saga", saga_id)

    async def _local_get_saga(self, saga_id: str) -> dict:
        orch = self.local._get_session(self._saga_session(saga_id)).saga
        return orch.get_saga(saga_id).to_dict()

    # -- agent-global views ----------------------------------------------------------------
    async def stats(self) -> dict:
        """X04: session / participant / saga / vouch totals over every rank."""
        return await self._view("stats")

    async def agent_ring(self, agent_did: str) -> Optional[dict]:
        """X05: the agent's ring in the earliest-created session where it is an
        active participant (reference: first match in ``_sessions`` order)."""
        return await self._view("agent_ring", agent_did)

    async def agent_liability(self, agent_did: str) -> dict:
        """The agent's vouches given/received on every rank in global vouch order;
        exposure = Σ live bonds given, summed in that order (bit-exact with one rank)."""
        return await self._view("agent_liability", agent_did)

    async def exposure_vector(self, agent_dids: list[str]) -> list[float]:
        """X01 dense: live bonded exposure of each agent over every rank's sessions —
        each rank reduces its store's edge columns on the device (K04), then one
        [A] fp64 all-reduce (RCCL over xGMI on MI355X)."""
        return await self._view("exposure_vector", list(agent_dids))

    async def list_sessions(self, state: Optional[str] = None) -> list[dict]:
        return await self._view("list_sessions", state)

    async def load(self) -> list[int]:
        """Sessions per rank."""
        return await self._view("load")

    async def _view(self, name: str, *args) -> Any:
        """Run a view on every member: rank 0 sequences them so all ranks enter the
        view's collectives in the same order."""
        self.counters["views"] += 1
        if self.world == 1:
            return self._combine(name, args, [self._collective(name, *args)])
        lead = self.members[0]
        if self.rank != lead:
            return await self.rpc.call(lead, "_view", name, *args)
        async with self._view_lock:
            others = [r for r in self.members if r != self.rank]
            for r in others:
                await self.rpc.connect(r)
            # the enter messages are written before this rank blocks in the collective
            peers = [self.rpc.send(r, "_view_enter", name, *args) for r in others]
            mine = self._collective(name, *args)
            parts = [mine] + list(await asyncio.gather(*peers))
        return self._combine(name, args, parts)

    def _collective(self, name: str, *args) -> Any:
        """This rank's part of a view (runs its collectives); JSON-serialisable."""
        hv = self.local
        if name == "stats":
            snaps = hv.snapshots()  # one batched device read
            sagas = hv.saga_summaries()
            vals = [len(snaps), sum(1 for x in snaps if x.state.value not in ("archived", "terminating")),
                    sum(x.participant_count for x in snaps),
                    sum(1 for g in sagas if g["state"] in ("running", "compensating")),
                    len(hv.vouching.records()), len(sagas)]
            t = torch.tensor(vals, dtype=torch.int64, device=_tensor_device())
            self._all_reduce(t, dist.ReduceOp.SUM)
            return [int(x) for x in t.tolist()]
        if name == "agent_ring":
            (agent_did,) = args
            big = (1 << 62) - 1
            best, sid = big, None
            for x in hv.snapshots(parts=True):
                for p in x.participants:
                    if p.agent_did == agent_did and p.is_active:
                        key = ((_us(x.created_at) - _EPOCH_US) << 12) | (self.rank << 4) | int(p.ring)
                        if key < best:
                            best, sid = key, x.session_id
                        break
            t = torch.tensor([best], dtype=torch.int64, device=_tensor_device())
            self._all_reduce(t, dist.ReduceOp.MIN)
            g = int(t.item())
            return [g, sid if g == best and g < big else None]
        if name == "agent_liability":
            (agent_did,) = args
            out = []
            for v in hv.vouching.records():
                if v.voucher_did == agent_did or v.vouchee_did == agent_did:
                    key = self._vouch_key.get(v.vouch_id, (_us(v.created_at), self.rank, 1 << 40))
                    out.append([list(key), _vouch_dict(v)])
            return out
        if name == "exposure_vector":
            (dids,) = args
            x = self._local_exposure(dids)
            self._all_reduce(x, dist.ReduceOp.SUM)
            return x.cpu().tolist()
        if name == "list_sessions":
            (state,) = args
            return [[_us(x.created_at), self.rank, i,
                     {"session_id": x.session_id, "state": x.state.value, "participant_count": x.participant_count,
                      "rank": self.rank}]
                    for i, x in enumerate(hv.snapshots()) if state is None or x.state.value == state]
        if name == "load":
            return len(hv.sessions)
        raise ValueError(f"unknown view {name!r}")

    def _combine(self, name: str, args, parts: list) -> Any:
        if name == "stats":
            keys = ("total_sessions", "active_sessions", "total_participants", "active_sagas", "total_vouches",
                    "total_sagas")
            return dict(zip(keys, parts[0]))
        if name == "agent_ring":
            g = parts[0][0]
            if g >= (1 << 62) - 1:
                return None
            sid = next(p[1] for p in parts if p[1] is not None)
            return {"agent_did": args[0], "ring": g & 0xF, "session_id": sid}
        if name == "agent_liability":
            agent_did = args[0]
            allv = sorted(((tuple(k), d) for part in parts for k, d in part), key=lambda r: r[0])
            given = [d for _, d in allv if d["voucher_did"] == agent_did]
            received = [d for _, d in allv if d["vouchee_did"] == agent_did]
            exposure = 0.0
            for d in given:
                if d["is_active"] and not d["is_expired"]:
                    exposure += d["bonded_amount"]
            return {"agent_did": agent_did, "vouches_given": given, "vouches_received": received,
                    "total_exposure": exposure}
        if name == "exposure_vector":
            return parts[0]
        if name == "list_sessions":
            rows = sorted((tuple(p[:3]), p[3]) for part in parts for p in part)
            return [d for _, d in rows]
        if name == "load":
            out = [0] * self.world
            for r, n in zip(self.members, parts):
                out[r] = n
            return out
        raise ValueError(name)

    def _local_exposure(self, dids: list[str]) -> torch.Tensor:
        """K04 over this rank's vouch edges: Σ live bonded amount per voucher, for
        the agents ``dids`` (dense, in that order), fp64 on the collective device."""
        dev = _tensor_device()
        hv = self.local
        st = hv._store
        if st is None:  # host engines
            idx = {d: i for i, d in enumerate(dids)}
            x = torch.zeros(len(dids), dtype=torch.float64)
            for v in hv.vouching.records():
                k = idx.get(v.voucher_did)
                if k is not None and v.is_live:
                    x[k] += v.bonded_amount
            return x.to(dev)
        from agent_hypervisor_amd.ops.store_views import exposure_by_agent

        return exposure_by_agent(st, [st.agents.lookup(d) for d in dids], list(hv.vouching._by_edge)).to(dev)

    def _all_reduce(self, t: torch.Tensor, op) -> None:
        if self.world > 1:
            self.counters["collectives"] += 1
            dist.all_reduce(t, op=op, group=self.data_group)

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
        """One failure verdict for all survivors: the first rank to claim the next
        failover epoch (an atomic counter in the rendezvous store) publishes its
        suspect list; every survivor — the claimant included — adopts the
        published list, so views that differ by a heartbeat cannot split the job."""
        from agent_hypervisor_amd.parallel.resilience import _store

        st = _store()
        key = f"ahv/failover/{len(self.failovers)}"
        if st.add(key + "/claim", 1) == 1:
            st.set(key, json.dumps(sorted(int(r) for r in suspects)))
        st.wait([key])
        return json.loads(st.get(key).decode())

    def checkpoint(self, root: str) -> str:
        """Each rank persists its own sessions and its share of the global vouch order
        under ``root/rank<r>`` (one atomic publish); collective over the members."""
        from agent_hypervisor_amd.runtime.checkpoint import save_hypervisor

        meta = {"rank": self.rank, "vouch_key": {k: list(v) for k, v in self._vouch_key.items()},
                "sagas": self._sagas}
        d = save_hypervisor(self.local, os.path.join(root, f"rank{self.rank}"),
                            extra_files={"sharded.json": json.dumps(meta)})
        if self.world > 1:
            dist.barrier(group=self.group)
        return d

    async def failover(self, failed: list[int], root: str) -> list[tuple[str, int, int]]:
        """Survivors (every remaining member calls this): drop the failed ranks,
        re-home their sessions and liability-only sessions with :meth:`owner` over
        the survivors, re-hydrate the ones this rank now owns from the failed
        ranks' checkpoints (audit chains re-verified on load), and move the
        collectives to sub-groups of the survivors."""
        from agent_hypervisor_amd.runtime.checkpoint import checkpoint_session_keys, load_hypervisor

        failed = sorted(set(failed) & set(self.members))
        if not failed:
            return []
        if self.rank in failed:
            raise RuntimeError("a failed rank cannot take part in its own failover")
        self.members = [r for r in self.members if r not in failed]
        self._live = frozenset(self.members)
        moves = []
        for f in failed:
            if self.rpc is not None:
                self.rpc.drop(f)
            src = os.path.join(root, f"rank{f}")
            keys = checkpoint_session_keys(src)  # hypervisor sessions + liability-only session ids
            moves.extend((k, f, self.owner(k)) for k in keys)
            mine = sorted(k for k in keys if self.owner(k) == self.rank)
            if mine:
                load_hypervisor(src, hv=self.local, sessions=mine)
            meta = os.path.join(src, "sharded.json")
            if os.path.exists(meta):
                with open(meta) as fh:
                    m = json.load(fh)
                mine_set = set(mine)
                self._sagas.update({g: s for g, s in m.get("sagas", {}).items() if s in mine_set})
                for vid, key in m.get("vouch_key", {}).items():
                    self._vouch_key.setdefault(vid, tuple(key))
        # only the survivors synchronise on these groups (the failed ranks never call in)
        self.group = dist.new_group(ranks=self.members, backend="gloo", use_local_synchronization=True)
        self.data_group = dist.new_group(ranks=self.members, use_local_synchronization=True)
        self.failovers.append({"failed": failed, "moves": len(moves)})
        return moves


def _vouch_dict(v) -> dict:
    return {
        "vouch_id": v.vouch_id, "voucher_did": v.voucher_did, "vouchee_did": v.vouchee_did,
        "session_id": v.session_id, "bonded_sigma_pct": v.bonded_sigma_pct, "bonded_amount": v.bonded_amount,
        "is_active": bool(v.is_active), "is_expired": bool(v.is_expired),
    }


async def serve_followers(shv: ShardedHypervisor) -> None:
    """Ranks ≠ 0 of a REST deployment: serve forwarded calls and views until the
    front-end rank shuts the job down."""
    await shv.serve_forever()
