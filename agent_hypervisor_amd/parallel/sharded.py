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
  ``GET /api/v1/stats`` (:145-163)         X04: each rank's counters reduced on
                                           the device over its rows (no snapshot
                                           per session), one 48-byte all-reduce
  ``GET /agents/{did}/ring`` (:319-331)    X05 all-reduce MIN of (creation time,
                                           rank, ring) keys
  ``GET /agents/{did}/liability`` (:570)   owner-routed (P02): the agent's owner
                                           rank gathers every rank's compact
                                           record set from its per-agent index
                                           point to point and sums exposure in
                                           global vouch order (bit-exact with
                                           one rank); no rank-0 sequencing
  dense per-agent exposure                 X01: K04 over each rank's store edge
                                           columns → [A] fp64 all-reduce
  ``GET /api/v1/sessions``                 per-rank snapshots, merged by creation
  ``GET /api/v1/events`` (:328-343)        each rank's event bus, merged by
                                           (timestamp, rank, sequence)
  ``GET /api/v1/events/stats`` (:346)      per-type counts summed over ranks
  =======================================  ======================================

  A view never stalls a rank's serving: its local part (batched device reads)
  runs on the event loop, its blocking collective on a dedicated communication
  thread (:attr:`ShardedHypervisor._comm`), so forwarded per-session calls keep
  completing on every rank while a view is in flight.  X05 (agent ring) is one
  device MIN over the store's participant columns of the rank's sessions (O(1)
  store commands); the agent-liability view gathers bond state from the edge
  columns in one read.
* **The rest of the per-session surface** routes the same way: ring
  distribution, saga and vouch listings, and the session object's operations —
  leave, ring updates, consistency mode, VFS write/read/delete/permissions and
  snapshot/restore (:meth:`ShardedHypervisor.sso`).

Failure handling: heartbeats, one agreed failure verdict (the first
proposer's list wins), checkpoints per rank, and failover — the dead rank's
sessions *and* liability-only sessions re-home deterministically (to the next
live rank after their home) and are re-hydrated from its checkpoint there.
"""

from __future__ import annotations

import asyncio
import json
import os
from concurrent.futures import ThreadPoolExecutor
from dataclasses import asdict
from datetime import datetime
from typing import Any, Callable, Optional

import torch
import torch.distributed as dist

from agent_hypervisor_amd.parallel.directory import stable_rank
from hypervisor.models import ConsistencyMode, SessionConfig

_CTRL: dict = {}


class ViewAborted(RuntimeError):
    """An agent-global view whose collective was abandoned by :meth:`ShardedHypervisor.failover`."""


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


async def _api_executor():
    return {"status": "executed_via_api"}  # what the reference REST step execution runs


# per-session methods served for other ranks (the RPC whitelist)
_SERVED = (
    "create_session", "join_session", "activate_session", "terminate_session", "verify_behavior", "get_session",
    "capture", "merkle_root", "vouch", "compute_sigma_eff", "get_total_exposure", "release_session_bonds",
    "slash", "create_saga", "add_step", "execute_step", "compensate", "get_saga",
    "ring_distribution", "list_sagas", "list_vouches", "sso",
    "agent_liability_owner", "liability_part", "dir_register",
    "_view", "_view_enter", "_stop",
)


def _edit(e) -> Optional[dict]:
    return None if e is None else {"path": e.path, "operation": e.operation, "agent_did": e.agent_did,
                                   "timestamp": e.timestamp.isoformat() if e.timestamp else None,
                                   "content_hash": e.content_hash, "previous_hash": e.previous_hash}


def _participant(p) -> dict:
    return {"agent_did": p.agent_did, "ring": int(p.ring), "sigma_raw": p.sigma_raw, "sigma_eff": p.sigma_eff,
            "joined_at": p.joined_at.isoformat() if p.joined_at else None, "is_active": p.is_active}


def _perms(p) -> Optional[list]:
    return None if p is None else sorted(p)


def _sso_ops() -> dict:
    from hypervisor.models import ExecutionRing

    # SharedSessionObject operations (reference session/__init__.py:115-175 and its VFS),
    # run on the owner; arguments and results are JSON values
    return {
        "leave": lambda s, did: s.leave(did),
        "update_ring": lambda s, did, ring: s.update_ring(did, ExecutionRing(ring)),
        "force_consistency_mode": lambda s, mode: s.force_consistency_mode(ConsistencyMode(mode)),
        "get_participant": lambda s, did: _participant(s.get_participant(did)),
        "vfs_write": lambda s, path, content, did: _edit(s.vfs.write(path, content, did)),
        "vfs_read": lambda s, path, did=None: s.vfs.read(path, did),
        "vfs_delete": lambda s, path, did: _edit(s.vfs.delete(path, did)),
        "vfs_list": lambda s: s.vfs.list_files(),
        "vfs_set_permissions": lambda s, path, agents, did: _edit(s.vfs.set_permissions(path, set(agents), did)),
        "vfs_get_permissions": lambda s, path: _perms(s.vfs.get_permissions(path)),
        "vfs_snapshot": lambda s, snapshot_id=None: s.create_vfs_snapshot(snapshot_id),
        "vfs_restore": lambda s, snapshot_id, did: s.restore_vfs_snapshot(snapshot_id, did),
        "vfs_list_snapshots": lambda s: s.vfs.list_snapshots(),
        "vfs_delete_snapshot": lambda s, snapshot_id: s.vfs.delete_snapshot(snapshot_id),
    }


_SSO: dict = {}


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
        if "event_bus" not in hv_kwargs:  # each rank publishes its own sessions' events
            from hypervisor.observability.event_bus import HypervisorEventBus

            hv_kwargs["event_bus"] = HypervisorEventBus()
        self.local = Hypervisor(device=device, **hv_kwargs)
        self.bus = self.local.event_bus
        self._comm: Optional[ThreadPoolExecutor] = None  # the communication thread of the views
        self._inflight: set = set()  # asyncio futures of view collectives running on that thread
        self.members = list(range(self.world))
        self._live = frozenset(self.members)
        self.group = None if self.world == 1 else control_group()
        self.data_group = None  # default group (RCCL on MI355X) until a failover
        self.rpc = None
        self.executors: dict[str, Callable[..., Any]] = {"noop": _noop, "api": _api_executor}
        self.compensators: dict[str, Callable[..., Any]] = {"noop": _noop_comp}
        self.counters = {"local": 0, "forwarded": 0, "collectives": 0, "views": 0, "liability_parts": 0,
                         "dir_registrations": 0}
        self._rr = 0
        self._sagas: dict[str, str] = {}  # saga id → session id (sagas this rank owns)
        self._vouch_seq = 0
        self._vouch_key: dict[str, tuple] = {}  # vouch id → global order key (created µs, rank, seq)
        self._moved: dict[str, int] = {}  # session / saga id → owner after a migration (same on every rank)
        self._agent_ix: dict[str, list] = {}  # agent DID → its vouch records on this rank (creation order)
        self._agent_ix_n = 0  # records the index covers
        # P02 owner-resident agent directory: on an agent's owner rank (owner(did)), the
        # members that hold vouch records naming it — agent_liability asks only those
        self._agent_dir: dict[str, set] = {}
        self._dir_sent: set = set()  # agents this rank has registered with their owner
        self._dir_ok = True  # False: liability views ask every member until the next rebuild
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
        self._drop_comm()

    def _drop_comm(self) -> None:
        """Abandon the views' communication thread without waiting for it: a
        collective still blocked on a group that lost a rank must not hold up
        shutdown or the next view (it ends when its backend times out)."""
        if self._comm is not None:
            self._comm.shutdown(wait=False, cancel_futures=True)
            self._comm = None

    async def _handle(self, name: str, args: list, kwargs: dict) -> Any:
        if name == "_stop":
            self._stopped.set()
            return True
        if name == "_view":
            return await self._view(*args)
        if name == "_view_enter":
            return await self._enter(*args)
        return await getattr(self, "_local_" + name)(*args, **kwargs)

    # -- placement ---------------------------------------------------------------------
    def owner(self, key: str) -> int:
        """Owner rank of a session / liability-session / saga id: its home — a stable
        hash over the world — or, when the home rank has failed, the next live rank
        after it.  Re-homing by home rank (not by key) keeps a saga with its session
        (their ids were minted for the same home) on every survivor's routing."""
        live = self._live
        m = self._moved.get(key)
        if m is not None and m in live:  # migrated (rebalance / retire): its current owner
            return m
        h = stable_rank(key, self.world)
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
    async def create_session(self, config: SessionConfig, creator_did: str, rank: Optional[int] = None,
                             detail: bool = False):
        """Create a session on ``rank`` (default: this rank with policy ``local``,
        the next live rank with ``round_robin``); returns its id (``detail``: the
        REST route's CreateSessionResponse fields)."""
        if rank is None:
            if self.policy == "local":
                rank = self.rank
            else:
                rank = self.members[self._rr % len(self.members)]
                self._rr += 1
        sid = self._mint("session:", rank)
        return await self._route(sid, "create_session", _cfg_out(config), creator_did, sid, detail)

    async def _local_create_session(self, cfg: dict, creator_did: str, sid: str, detail: bool = False):
        m = await self.local.create_session(_cfg_in(cfg), creator_did, session_id=sid)
        if not detail:
            return m.sso.session_id
        x = m.sso
        return {"session_id": x.session_id, "state": x.state.value, "consistency_mode": x.consistency_mode.value,
                "created_at": x.created_at.isoformat()}

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

    async def get_session(self, session_id: str, detail: bool = False) -> dict:
        """Session summary (``detail``: the REST route's SessionDetailResponse fields)."""
        return await self._route(session_id, "get_session", session_id, detail)

    async def _local_get_session(self, session_id: str, detail: bool = False) -> dict:
        m = self.local.get_session(session_id)
        if m is None:
            raise ValueError(f"Session {session_id} not found")
        if detail:
            from hypervisor.api.models import ParticipantInfo

            sso = m.sso
            return {"session_id": sso.session_id, "state": sso.state.value,
                    "consistency_mode": sso.consistency_mode.value, "creator_did": sso.creator_did,
                    "participant_count": sso.participant_count,
                    "participants": [ParticipantInfo.of(p).model_dump() for p in sso.participants],
                    "created_at": sso.created_at.isoformat(),
                    "terminated_at": sso.terminated_at.isoformat() if sso.terminated_at else None,
                    "sagas": [g.to_dict() for g in m.saga.sagas]}
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
                    bond_pct: Optional[float] = None, expiry: Optional[datetime] = None, emit: bool = False) -> dict:
        """``emit``: publish the REST route's ``vouch.created`` event on the owner."""
        return await self._route(session_id, "vouch", voucher_did, vouchee_did, session_id, voucher_sigma, bond_pct,
                                 expiry.isoformat() if expiry is not None else None, emit)

    async def _local_vouch(self, voucher_did, vouchee_did, session_id, voucher_sigma, bond_pct=None, expiry=None,
                           emit: bool = False):
        exp = datetime.fromisoformat(expiry) if expiry else None
        v = self.local.vouching.vouch(voucher_did, vouchee_did, session_id, voucher_sigma, bond_pct, exp)
        self._vouch_seq += 1
        self._vouch_key[v.vouch_id] = (_us(v.created_at), self.rank, self._vouch_seq)
        self._index_vouch(v)
        await self._dir_note(voucher_did, vouchee_did)
        if emit:  # the REST route's event (reference api/server.py vouch handler)
            from hypervisor.observability.event_bus import EventType

            self.local._emit(EventType.VOUCH_CREATED, session_id, voucher_did, vouch_id=v.vouch_id,
                             vouchee_did=vouchee_did, bonded_amount=v.bonded_amount)
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
    async def create_saga(self, session_id: str, emit: bool = False):
        """Returns the saga id (``emit``: the REST route's form — its event is
        published on the owner and the CreateSagaResponse fields returned)."""
        gid = self._mint("saga:", self.owner(session_id))
        return await self._route(session_id, "create_saga", session_id, gid, emit)

    async def _local_create_saga(self, session_id: str, gid: str, emit: bool = False):
        g = self.local._get_session(session_id).saga.create_saga(session_id, saga_id=gid)
        self._sagas[gid] = session_id
        if not emit:
            return gid
        from hypervisor.observability.event_bus import EventType

        self.local._emit(EventType.SAGA_CREATED, session_id, saga_id=gid)
        return {"saga_id": gid, "session_id": g.session_id, "state": g.state.value,
                "created_at": g.created_at.isoformat()}

    def _saga_session(self, saga_id: str) -> str:
        sid = self._sagas.get(saga_id)
        if sid is None:
            from hypervisor.saga.state_machine import SagaStateError

            raise SagaStateError(f"Saga {saga_id} not found")
        return sid

    async def add_step(self, saga_id: str, action_id: str, agent_did: str, execute_api: str,
                       undo_api: Optional[str] = None, timeout_seconds: int = 300, max_retries: int = 0,
                       detail: bool = False):
        """Returns the step id (``detail``: the REST route's AddStepResponse fields;
        a refused step then raises RuntimeError — the route's 400)."""
        return await self._route(saga_id, "add_step", saga_id, action_id, agent_did, execute_api, undo_api,
                                 timeout_seconds, max_retries, detail)

    async def _local_add_step(self, saga_id, action_id, agent_did, execute_api, undo_api=None, timeout_seconds=300,
                              max_retries=0, detail: bool = False):
        orch = self.local._get_session(self._saga_session(saga_id)).saga
        if not detail:
            return orch.add_step(saga_id, action_id, agent_did, execute_api, undo_api, timeout_seconds,
                                 max_retries).step_id
        try:
            st = orch.add_step(saga_id, action_id, agent_did, execute_api, undo_api, timeout_seconds, max_retries)
        except Exception as e:  # noqa: BLE001 - the single-rank route answers 400
            raise RuntimeError(str(e)) from e
        return {"step_id": st.step_id, "saga_id": saga_id, "action_id": st.action_id, "state": st.state.value}

    def register_executor(self, name: str, fn: Callable[..., Any]) -> None:
        """Make an executor callable by name from any rank (register on every rank)."""
        self.executors[name] = fn

    def register_compensator(self, name: str, fn: Callable[..., Any]) -> None:
        self.compensators[name] = fn

    async def execute_step(self, saga_id: str, step_id: str, executor: Any = "noop", rest: bool = False) -> Any:
        """``executor``: a registered name (any rank) or a callable (owner rank only).
        ``rest``: the REST route's form — failures are reported, not raised, as
        ``{"state", "error"}``, with the route's step event published on the owner."""
        if callable(executor):
            if self.owner(saga_id) != self.rank:
                raise TypeError("executors cross ranks by name: register_executor() on every rank")
            self.counters["local"] += 1
            return await self._exec_step(saga_id, step_id, executor)
        return await self._route(saga_id, "execute_step", saga_id, step_id, executor, rest)

    async def _local_execute_step(self, saga_id: str, step_id: str, executor: str = "noop", rest: bool = False) -> Any:
        fn = self.executors.get(executor)
        if fn is None:
            raise KeyError(f"executor {executor!r} is not registered on rank {self.rank}")
        if not rest:
            return await self._exec_step(saga_id, step_id, fn)
        from hypervisor.observability.event_bus import EventType

        sid = self._saga_session(saga_id)
        orch = self.local._get_session(sid).saga
        saga = orch.get_saga(saga_id)
        if saga is None or not any(x.step_id == step_id for x in saga.steps):
            raise ValueError(f"Saga {saga_id} or step {step_id} not found")
        try:
            await orch.execute_step(saga_id, step_id, executor=fn)
        except Exception as e:  # noqa: BLE001 - the single-rank route answers 400
            raise RuntimeError(str(e)) from e
        for x in saga.steps:
            if x.step_id == step_id:
                et = EventType.SAGA_STEP_COMMITTED if x.state.value == "committed" else EventType.SAGA_STEP_FAILED
                self.local._emit(et, saga.session_id, x.agent_did, saga_id=saga_id, step_id=step_id)
                return {"state": x.state.value, "error": x.error}
        raise ValueError(f"Saga {saga_id} or step {step_id} not found")

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

    async def get_saga(self, saga_id: str, detail: bool = False) -> dict:
        """``saga.to_dict()`` (``detail``: the REST route's SagaDetailResponse fields)."""
        return await self._route(saga_id, "get_saga", saga_id, detail)

    async def _local_get_saga(self, saga_id: str, detail: bool = False) -> dict:
        orch = self.local._get_session(self._saga_session(saga_id)).saga
        if detail:
            from hypervisor.api.models import SagaDetailResponse

            return SagaDetailResponse.of(orch.get_saga(saga_id)).model_dump()
        return orch.get_saga(saga_id).to_dict()

    # -- the rest of the per-session surface (reference api/server.py:192-309) ------------
    async def ring_distribution(self, session_id: str) -> dict:
        """``GET /sessions/{id}/rings``: ring name → participant DIDs."""
        return await self._route(session_id, "ring_distribution", session_id)

    async def _local_ring_distribution(self, session_id: str) -> dict:
        out: dict = {}
        for p in self.local._get_session(session_id).sso.participants:
            out.setdefault(p.ring.name, []).append(p.agent_did)
        return out

    def check_ring(self, agent_ring: int, action: dict, sigma_eff: float, has_consensus: bool = False,
                   has_sre_witness: bool = False) -> dict:
        """``POST /rings/check``: stateless, answered by the calling rank."""
        from hypervisor.models import ActionDescriptor, ExecutionRing

        r = self.local.ring_enforcer.check(agent_ring=ExecutionRing(agent_ring), action=ActionDescriptor(**action),
                                           sigma_eff=sigma_eff, has_consensus=has_consensus,
                                           has_sre_witness=has_sre_witness)
        return {"allowed": r.allowed, "required_ring": r.required_ring.value, "agent_ring": r.agent_ring.value,
                "sigma_eff": r.sigma_eff, "reason": r.reason, "requires_consensus": r.requires_consensus,
                "requires_sre_witness": r.requires_sre_witness}

    async def list_sagas(self, session_id: str) -> list:
        """``GET /sessions/{id}/sagas`` (SagaDetailResponse rows)."""
        return await self._route(session_id, "list_sagas", session_id)

    async def _local_list_sagas(self, session_id: str) -> list:
        from hypervisor.api.models import SagaDetailResponse

        return [SagaDetailResponse.of(g).model_dump() for g in self.local._get_session(session_id).saga.sagas]

    async def list_vouches(self, session_id: str) -> list:
        """``GET /sessions/{id}/vouches`` (VouchResponse rows, creation order)."""
        return await self._route(session_id, "list_vouches", session_id)

    async def _local_list_vouches(self, session_id: str) -> list:
        from hypervisor.api.models import VouchResponse

        self.local._get_session(session_id)  # unknown session: 404 like the single-rank route
        return [VouchResponse.of(v).model_dump() for v in self.local.vouching.records(session_id)]

    async def sso(self, session_id: str, op: str, *args) -> Any:
        """A SharedSessionObject operation on the session's owner: ``leave``,
        ``update_ring``, ``force_consistency_mode``, ``get_participant``,
        ``vfs_write`` / ``vfs_read`` / ``vfs_delete`` / ``vfs_list``,
        ``vfs_set_permissions`` / ``vfs_get_permissions``, ``vfs_snapshot`` /
        ``vfs_restore`` / ``vfs_list_snapshots`` / ``vfs_delete_snapshot``."""
        return await self._route(session_id, "sso", session_id, op, *args)

    async def _local_sso(self, session_id: str, op: str, *args) -> Any:
        if not _SSO:
            _SSO.update(_sso_ops())
        fn = _SSO.get(op)
        if fn is None:
            raise ValueError(f"unknown session operation {op!r}")
        return fn(self.local._get_session(session_id).sso, *args)

    async def leave_session(self, session_id: str, agent_did: str) -> None:
        await self.sso(session_id, "leave", agent_did)

    async def update_ring(self, session_id: str, agent_did: str, ring: int) -> None:
        await self.sso(session_id, "update_ring", agent_did, int(ring))

    async def vfs_write(self, session_id: str, path: str, content: str, agent_did: str) -> dict:
        return await self.sso(session_id, "vfs_write", path, content, agent_did)

    async def vfs_read(self, session_id: str, path: str, agent_did: Optional[str] = None) -> Optional[str]:
        return await self.sso(session_id, "vfs_read", path, agent_did)

    async def vfs_delete(self, session_id: str, path: str, agent_did: str) -> dict:
        return await self.sso(session_id, "vfs_delete", path, agent_did)

    async def vfs_snapshot(self, session_id: str, snapshot_id: Optional[str] = None) -> str:
        return await self.sso(session_id, "vfs_snapshot", snapshot_id)

    async def vfs_restore(self, session_id: str, snapshot_id: str, agent_did: str) -> None:
        await self.sso(session_id, "vfs_restore", snapshot_id, agent_did)

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
        exposure = Σ live bonds given, summed in that order (bit-exact with one rank).

        Owner-routed (P02): the agent's owner rank — a stable hash of its DID over
        the live ranks — keeps the agent's directory entry (the members holding vouch
        records that name it, registered once per agent and holding rank by the
        vouch itself, rebuilt after migration / restore / failover) and asks only
        those members for their compact record sets (point to point, no collective,
        no rank-0 sequencing), then combines them.  Each rank answers from its
        per-agent vouch index (O(the agent's records), never a scan of all vouches)
        with bond state from one gather of the store's edge columns."""
        self.counters["views"] += 1
        o = self.owner(agent_did)
        if o == self.rank:
            return await self._local_agent_liability_owner(agent_did)
        self.counters["forwarded"] += 1
        return await self.rpc.call(o, "agent_liability_owner", agent_did)

    async def _local_agent_liability_owner(self, agent_did: str) -> dict:
        parts = [self._local_liability(agent_did)]
        if self._dir_ok:  # the members the directory lists (none: the agent has no records elsewhere)
            others = [r for r in sorted(self._agent_dir.get(agent_did, ())) if r != self.rank and r in self._live]
        else:
            others = [r for r in self.members if r != self.rank]
        if others:
            self.counters["liability_parts"] += len(others)
            parts += await asyncio.gather(*[self.rpc.call(r, "liability_part", agent_did) for r in others])
        return self._combine("agent_liability", (agent_did,), parts)

    # -- P02 agent directory (owner-resident) -----------------------------------------------
    async def _dir_note(self, *dids: str) -> None:
        """Register this rank with the owner of each agent the first time it holds a
        vouch record naming it — awaited, so a liability view issued after the vouch
        returns finds this rank listed.  One message per (agent, holding rank), not
        one per view; records that arrive by migration, restore or failover are
        covered by :meth:`_dir_rebuild`."""
        if self.world == 1:
            return
        for did in dids:
            if did in self._dir_sent:
                continue
            o = self.owner(did)
            if o == self.rank:
                self._agent_dir.setdefault(did, set()).add(self.rank)
            else:
                self.counters["dir_registrations"] += 1
                await self.rpc.call(o, "dir_register", did, self.rank)
            self._dir_sent.add(did)

    async def _local_dir_register(self, did: str, rank: int) -> bool:
        self._agent_dir.setdefault(did, set()).add(int(rank))
        return True

    def _dir_rebuild(self) -> None:
        """Collective over the members: the directory from every member's own records
        (after records moved between ranks or the owners changed: migration, restore,
        failover).  Each member sends the agents its records name; each keeps the
        entries of the agents it owns."""
        if self.world == 1 or len(self.members) == 1:
            self._agent_dir, self._dir_sent, self._dir_ok = {}, set(), True
            return
        from agent_hypervisor_amd.parallel import migrate as MG

        self._agent_records("")  # refresh the per-agent index
        mine = sorted(self._agent_ix)
        allm = MG.all_gather_json(mine, len(self.members), group=self.group)
        d: dict = {}
        for r, agents in zip(self.members, allm):
            for a in agents:
                if self.owner(a) == self.rank:
                    d.setdefault(a, set()).add(int(r))
        self._agent_dir, self._dir_sent, self._dir_ok = d, set(mine), True

    async def _local_liability_part(self, agent_did: str) -> list:
        return self._local_liability(agent_did)

    async def exposure_vector(self, agent_dids: list[str]) -> list[float]:
        """X01 dense: live bonded exposure of each agent over every rank's sessions —
        each rank reduces its store's edge columns on the device (K04), then one
        [A] fp64 all-reduce (RCCL over xGMI on MI355X)."""
        return await self._view("exposure_vector", list(agent_dids))

    async def list_sessions(self, state: Optional[str] = None) -> list[dict]:
        return await self._view("list_sessions", state)

    async def events(self, event_type: Optional[str] = None, session_id: Optional[str] = None,
                     agent_did: Optional[str] = None, limit: Optional[int] = None) -> list[dict]:
        """``GET /events``: every rank's bus filtered, merged by (timestamp, rank,
        sequence); ``limit`` keeps the latest ones (reference event_bus.py:158-175)."""
        return await self._view("events", event_type, session_id, agent_did, limit)

    async def event_stats(self) -> dict:
        """``GET /events/stats``: total and per-type counts over every rank."""
        return await self._view("event_stats")

    async def hold(self, seconds: float) -> int:
        """Diagnostics view: every rank keeps its collective open ``seconds`` (what a
        slow view looks like); per-session calls keep being served meanwhile."""
        return await self._view("hold", float(seconds))

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
            # every rank enters; this rank's collective runs on its communication thread
            peers = [self.rpc.send(r, "_view_enter", name, *args) for r in others]
            mine = await self._enter(name, *args)
            parts = [mine] + list(await asyncio.gather(*peers))
        return self._combine(name, args, parts)

    async def _enter(self, name: str, *args) -> Any:
        """This rank's part of a view: the local reads on the event loop (the store
        is not shared across threads), the blocking collective on the
        communication thread — the loop keeps serving per-session calls while the
        collective waits for the other ranks — then the JSON answer."""
        part, t, op, wait_s = self._local_part(name, *args)
        if t is not None and (self.world > 1 or wait_s):
            if self._comm is None:
                self._comm = ThreadPoolExecutor(max_workers=1, thread_name_prefix="ahv-comm")
            fut = asyncio.get_running_loop().run_in_executor(self._comm, self._blocking_collective, t, op, wait_s)
            self._inflight.add(fut)
            try:
                await fut
            except asyncio.CancelledError:
                if fut.cancelled():  # failover() abandoned it: the group lost a member
                    raise ViewAborted(f"view {name!r} aborted: a member failed while its collective was open") \
                        from None
                raise
            finally:
                self._inflight.discard(fut)
        return self._finish(name, args, part, t)

    def _blocking_collective(self, t: torch.Tensor, op, wait_s: float) -> None:
        if wait_s:
            import time

            time.sleep(wait_s)
        self._all_reduce(t, op)

    def _collective(self, name: str, *args) -> Any:
        """Synchronous form of :meth:`_enter` (one-rank façades)."""
        part, t, op, _ = self._local_part(name, *args)
        if t is not None:
            self._all_reduce(t, op)
        return self._finish(name, args, part, t)

    def _local_part(self, name: str, *args) -> tuple:
        """(local data, tensor to all-reduce or None, reduce op, hold seconds)."""
        hv = self.local
        dev = _tensor_device()
        if name == "stats":
            # device counters over the rank's rows (one reduction, no snapshot per
            # session), then the 48-byte X04 all-reduce
            c = hv.counters()
            vals = [c[k] for k in _STAT_KEYS]
            return None, torch.tensor(vals, dtype=torch.int64, device=dev), dist.ReduceOp.SUM, 0.0
        if name == "agent_ring":
            (agent_did,) = args
            best, sid = self._local_first_ring(agent_did)
            return (best, sid), torch.tensor([best], dtype=torch.int64, device=dev), dist.ReduceOp.MIN, 0.0
        if name == "exposure_vector":
            (dids,) = args
            return None, self._local_exposure(dids), dist.ReduceOp.SUM, 0.0
        if name == "list_sessions":
            (state,) = args
            return [[_us(x.created_at), self.rank, i,
                     {"session_id": x.session_id, "state": x.state.value, "consistency_mode": x.consistency_mode.value,
                      "participant_count": x.participant_count, "created_at": x.created_at.isoformat(),
                      "rank": self.rank}]
                    for i, x in enumerate(hv.snapshots()) if state is None or x.state.value == state], None, None, 0.0
        if name == "load":
            return len(hv.sessions), None, None, 0.0
        if name == "events":
            et, sid, did, limit = args
            from hypervisor.observability.event_bus import EventType

            bus = self.bus
            if bus is None:
                return [], None, None, 0.0
            evs = bus.query(event_type=EventType(et) if et else None, session_id=sid, agent_did=did)
            seq = {id(e): k for k, e in enumerate(bus.all_events)} if evs else {}
            if limit is not None:
                evs = evs[-int(limit):] if int(limit) > 0 else []
            return [[_us(e.timestamp), self.rank, seq[id(e)],
                     {"event_id": e.event_id, "event_type": e.event_type.value, "timestamp": e.timestamp.isoformat(),
                      "session_id": e.session_id, "agent_did": e.agent_did, "causal_trace_id": e.causal_trace_id,
                      "payload": e.payload}] for e in evs], None, None, 0.0
        if name == "event_stats":
            bus = self.bus
            return ({"total_events": bus.event_count if bus else 0, "by_type": bus.type_counts() if bus else {}},
                    None, None, 0.0)
        if name == "hold":
            (secs,) = args
            return None, torch.zeros(1, dtype=torch.int64, device=dev), dist.ReduceOp.SUM, float(secs)
        raise ValueError(f"unknown view {name!r}")

    def _finish(self, name: str, args, part, t) -> Any:
        if name in ("stats",):
            return [int(x) for x in t.tolist()]
        if name == "agent_ring":
            best, sid = part
            g = int(t.item())
            return [g, sid if g == best and g < _NO_RING else None]
        if name == "exposure_vector":
            return t.cpu().tolist()
        if name == "hold":
            return self.world
        return part

    def _local_first_ring(self, agent_did: str) -> tuple:
        """X05 on this rank: the key ((created − epoch) << 12 | rank << 4 | ring) of the
        earliest-created session (session order on ties) where the agent is an
        active participant, and that session's id.  Device-backed: one MIN over
        the store's participant columns of the rank's session rows."""
        hv = self.local
        st = hv._store
        if st is None:  # host engines: the snapshots in creation order
            return self._earliest(agent_did)
        from agent_hypervisor_amd.ops.store_views import first_active_ring, session_rows

        slots, sid_of = session_rows(hv)
        a = st.agents.lookup(agent_did)
        if a < 0 or not len(slots):
            return _NO_RING, None
        hit = first_active_ring(st, slots, a)
        if hit is None:
            return _NO_RING, None
        i, created, ring = hit
        return ((created - _EPOCH_US) << 12) | (self.rank << 4) | ring, sid_of(i)

    def _earliest(self, agent_did: str) -> tuple:
        """(key, session id) by a walk over the snapshots (creation order: the first
        match wins ties)."""
        best, sid = _NO_RING, None
        for x in self.local.snapshots(parts=True):
            for p in x.participants:
                if p.agent_did == agent_did and p.is_active:
                    key = ((_us(x.created_at) - _EPOCH_US) << 12) | (self.rank << 4) | int(p.ring)
                    if key < best:
                        best, sid = key, x.session_id
                    break
        return best, sid

    def _agent_records(self, agent_did: str) -> list:
        """This rank's vouch records naming the agent (voucher or vouchee), in
        creation order, from the per-agent index (rebuilt in one pass whenever
        records arrived by another path: checkpoint re-hydration, migration)."""
        recs = self.local.vouching.records()
        if self._agent_ix_n != len(recs):
            ix: dict = {}
            for v in recs:
                ix.setdefault(v.voucher_did, []).append(v)
                if v.vouchee_did != v.voucher_did:
                    ix.setdefault(v.vouchee_did, []).append(v)
            self._agent_ix, self._agent_ix_n = ix, len(recs)
        return self._agent_ix.get(agent_did, [])

    def _index_vouch(self, v) -> None:
        if self._agent_ix_n == len(self.local.vouching.records()) - 1:
            self._agent_ix.setdefault(v.voucher_did, []).append(v)
            if v.vouchee_did != v.voucher_did:
                self._agent_ix.setdefault(v.vouchee_did, []).append(v)
            self._agent_ix_n += 1

    def _local_liability(self, agent_did: str) -> list:
        """This rank's compact record set for the agent: ``[created µs, rank, seq,
        vouch id, voucher, vouchee, session id, bond pct, bonded, active, expired]``
        per record; bond state for all of them from one gather of the edge columns."""
        hv = self.local
        recs = self._agent_records(agent_did)
        st = hv._store
        state = {}
        if st is not None:
            live = [v.edge for v in recs if getattr(v, "edge", -1) >= 0]
            if live:
                g = st.gather({"e_active": live})
                state = {e: bool(a) for e, a in zip(live, g["e_active"].tolist())}
        out = []
        for v in recs:
            key = self._vouch_key.get(v.vouch_id, (_us(v.created_at), self.rank, 1 << 40))
            act = state.get(getattr(v, "edge", -1)) if st is not None else None
            out.append([*key, v.vouch_id, v.voucher_did, v.vouchee_did, v.session_id, v.bonded_sigma_pct,
                        v.bonded_amount, int(bool(v.is_active) if act is None else act), int(bool(v.is_expired))])
        return out

    def _combine(self, name: str, args, parts: list) -> Any:
        if name == "events":
            limit = args[3]
            rows = sorted((tuple(p[:3]), p[3]) for part in parts for p in part)
            out = [d for _, d in rows]
            if limit is not None:
                out = out[-int(limit):] if int(limit) > 0 else []
            return out
        if name == "event_stats":
            total, by = 0, {}
            for p in parts:
                total += p["total_events"]
                for k, v in p["by_type"].items():
                    by[k] = by.get(k, 0) + v
            return {"total_events": total, "by_type": by}
        if name == "hold":
            return parts[0]
        if name == "stats":
            return dict(zip(_STAT_KEYS, parts[0]))
        if name == "agent_ring":
            g = parts[0][0]
            if g >= (1 << 62) - 1:
                return None
            sid = next(p[1] for p in parts if p[1] is not None)
            return {"agent_did": args[0], "ring": g & 0xF, "session_id": sid}
        if name == "agent_liability":
            agent_did = args[0]
            allv = sorted(((tuple(r[:3]), _compact_vouch(r)) for part in parts for r in part), key=lambda r: r[0])
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

    # -- migration: rebalance and planned leave, no files -------------------
    def migrate(self, moves: dict) -> dict:
        """Collective over the members (every member calls, each with the moves of
        sessions *it* owns: ``{session_id: destination rank}``): the sessions —
        rows, chains with their records, sagas, steps, vouch bonds, commitments,
        extras — move device to device (:mod:`agent_hypervisor_amd.parallel.migrate`;
        RCCL ``all_to_all`` over xGMI on MI355X), their sagas and global vouch
        order keys with them, and every member routes them to their new owner
        afterwards.  Serving pauses on every member while it runs.  Returns
        ``{"sent", "received"}`` for this rank."""
        from agent_hypervisor_amd.parallel import migrate as MG

        if self.world == 1 or len(self.members) == 1:
            return {"sent": 0, "received": 0}
        hv = self.local
        bad = [s for s, d in moves.items() if d not in self._live or hv.get_session(s) is None]
        if bad:
            raise ValueError(f"cannot move {bad[:3]}: unknown here or destination not a live member")
        moves = {s: int(d) for s, d in moves.items() if int(d) != self.rank}
        by_sess: dict = {}
        for g, sid in self._sagas.items():
            if sid in moves:
                by_sess.setdefault(sid, []).append(g)
        vkeys = {v.vouch_id: list(self._vouch_key[v.vouch_id]) for v in hv.vouching.records()
                 if v.session_id in moves and v.vouch_id in self._vouch_key}
        mine = {"keys": {**moves, **{g: moves[s] for s, gs in by_sess.items() for g in gs}},
                "sagas": {g: s for s, gs in by_sess.items() for g in gs}, "vouch_key": vkeys,
                "dst": moves}
        allm = MG.all_gather_json(mine, len(self.members), group=self.group)
        plan: dict = {}
        for s_, d in moves.items():
            plan.setdefault(d, []).append(s_)
        got = MG.exchange(hv, plan, self.rank, self.members, ctrl_group=self.group, data_group=self.data_group)
        MG.evict(hv, list(moves))
        for m in allm:  # every member: the new routes; receivers: the moved sessions' sagas and vouch keys
            self._moved.update({k: int(v) for k, v in m["keys"].items()})
            for g, sid in m["sagas"].items():
                if int(m["dst"][sid]) == self.rank:
                    self._sagas[g] = sid
            for vid, key in m["vouch_key"].items():
                self._vouch_key[vid] = tuple(key)
        for g in [g for g, sid in self._sagas.items() if sid in moves]:
            del self._sagas[g]
        self._agent_ix_n = -1  # the per-agent vouch index is rebuilt on next use
        self._dir_rebuild()  # the moved records' holders, at their agents' owners
        self.counters["migrations"] = self.counters.get("migrations", 0) + 1
        return {"sent": len(moves), "received": len(got)}

    def rebalance(self) -> dict:
        """Collective: even out the members' session counts (within one session of
        the mean) by moving sessions from the most loaded members (their newest
        sessions) — :meth:`migrate` under a plan every member computes alike."""
        from agent_hypervisor_amd.parallel import migrate as MG

        if self.world == 1 or len(self.members) == 1:
            return {"sent": 0, "received": 0}
        loads_m = MG.all_gather_json(len(self.local._sessions), len(self.members), group=self.group)
        loads = {r: n for r, n in zip(self.members, loads_m)}
        moves: dict = {}
        ids = None
        for src, dst, c in MG.balance_plan(loads, self.members):
            if src != self.rank:
                continue
            if ids is None:
                ids = [s for s in self.local._sessions if s not in moves]
            take, ids = ids[-c:], ids[:-c]
            moves.update(dict.fromkeys(take, dst))
        return self.migrate(moves)

    def retire(self, rank: int) -> dict:
        """Collective: planned leave of member ``rank`` without checkpoint files —
        its sessions move to the other members (round robin, :meth:`migrate`), then
        every member drops it and the collectives move to sub-groups of the rest
        (crash failover, where the rank cannot send, still re-hydrates from its
        checkpoint: :meth:`failover`)."""
        if rank not in self.members or len(self.members) == 1:
            raise ValueError(f"rank {rank} is not a member that can leave {self.members}")
        rest = [r for r in self.members if r != rank]
        moves = {}
        if self.rank == rank:
            moves = {s: rest[i % len(rest)] for i, s in enumerate(list(self.local._sessions))}
        out = self.migrate(moves)
        self.members = rest
        self._live = frozenset(rest)
        if self.rank != rank:
            if self.rpc is not None:
                self.rpc.drop(rank)
            self._drop_comm()
            self.group = dist.new_group(ranks=self.members, backend="gloo", use_local_synchronization=True)
            self.data_group = dist.new_group(ranks=self.members, use_local_synchronization=True)
            self._dir_rebuild()  # agents homed on the leaver have new owners
        return out

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
                "sagas": self._sagas, "moved": self._moved, "members": self.members}
        d = save_hypervisor(self.local, os.path.join(root, f"rank{self.rank}"),
                            extra_files={"sharded.json": json.dumps(meta)})
        if self.world > 1:
            dist.barrier(group=self.group)
        return d

    def restore(self, root: str) -> int:
        """Collective: every rank re-loads its own ``root/rank<r>`` checkpoint (audit
        chains re-verified) and the job's routing state saved with it — saga homes,
        global vouch order keys and the routes of migrated sessions, so a session
        moved by :meth:`rebalance` / :meth:`retire` before the checkpoint still
        resolves to the rank that holds its rows.  Returns the sessions loaded here."""
        from agent_hypervisor_amd.runtime.checkpoint import load_hypervisor

        src = os.path.join(root, f"rank{self.rank}")
        n0 = len(self.local._sessions)
        load_hypervisor(src, hv=self.local)
        meta = os.path.join(src, "sharded.json")
        if os.path.exists(meta):
            with open(meta) as fh:
                m = json.load(fh)
            self._sagas.update(m.get("sagas", {}))
            for vid, key in m.get("vouch_key", {}).items():
                self._vouch_key.setdefault(vid, tuple(key))
            self._moved.update({k: int(v) for k, v in m.get("moved", {}).items()})
        self._agent_ix_n = -1
        if self.world > 1:
            dist.barrier(group=self.group)
        self._dir_rebuild()
        return len(self.local._sessions) - n0

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
                for k, v in m.get("moved", {}).items():  # routes of migrated ids (same on every rank)
                    self._moved.setdefault(k, int(v))
        # only the survivors synchronise on these groups (the failed ranks never call in);
        # a view collective still blocked on the old group stays on the old thread, and the
        # next view gets a fresh communication thread bound to the new groups
        for fut in list(self._inflight):  # their callers get ViewAborted instead of waiting on the old group
            fut.cancel()
        self._drop_comm()
        self.group = dist.new_group(ranks=self.members, backend="gloo", use_local_synchronization=True)
        self.data_group = dist.new_group(ranks=self.members, use_local_synchronization=True)
        self._agent_ix_n = -1
        self._dir_rebuild()  # re-homed records and the failed ranks' agents, at their new owners
        self.failovers.append({"failed": failed, "moves": len(moves)})
        return moves


_NO_RING = (1 << 62) - 1
_STAT_KEYS = ("total_sessions", "active_sessions", "total_participants", "active_sagas", "total_vouches",
              "total_sagas")


def _compact_vouch(r: list) -> dict:
    """A compact record of :meth:`ShardedHypervisor._local_liability` as the route's dict."""
    return {"vouch_id": r[3], "voucher_did": r[4], "vouchee_did": r[5], "session_id": r[6],
            "bonded_sigma_pct": r[7], "bonded_amount": r[8], "is_active": bool(r[9]), "is_expired": bool(r[10])}


def _vouch_dict(v, active: Optional[bool] = None) -> dict:
    """``active``: the bond state already gathered from the edge columns (None: ask the record)."""
    return {
        "vouch_id": v.vouch_id, "voucher_did": v.voucher_did, "vouchee_did": v.vouchee_did,
        "session_id": v.session_id, "bonded_sigma_pct": v.bonded_sigma_pct, "bonded_amount": v.bonded_amount,
        "is_active": bool(v.is_active) if active is None else active, "is_expired": bool(v.is_expired),
    }


async def serve_followers(shv: ShardedHypervisor) -> None:
    """Ranks ≠ 0 of a REST deployment: serve forwarded calls and views until the
    front-end rank shuts the job down."""
    await shv.serve_forever()
