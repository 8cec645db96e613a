"""REST front-end of the sharded (one process per GPU) hypervisor.

Any rank may serve HTTP (typically rank 0, or one front-end per rank behind a
load balancer).  Per-session routes run on the session's owner rank — directly
when this rank owns it, otherwise forwarded point-to-point to the owner while
the other ranks keep serving (:class:`~agent_hypervisor_amd.parallel.sharded.ShardedHypervisor`);
requests are handled concurrently.  The cross-session routes combine every rank
(``/stats`` X04, ``/agents/{did}/ring`` X05, ``/agents/{did}/liability`` X01,
``/sessions``, ``/events``, ``/events/stats``).  Ranks without a front-end run
:func:`~agent_hypervisor_amd.parallel.sharded.serve_followers`.  Error mapping
follows the single-process server (reference api/server.py): ``ValueError`` /
unknown ids → 404, other failures → 400.  The same routes, paths and request
bodies as :mod:`hypervisor.api.server` for every reference route (lifecycle,
rings, liability, sagas, events); each rank publishes its own sessions' events
and the events routes merge them.  The step executor of ``.../execute`` is the
registered ``"api"`` executor (the reference REST executes a no-op returning
``{"status": "executed_via_api"}``).  Responses use the single-process
server's response models, so each answer has the same shape and values.
"""

from __future__ import annotations

from typing import Any, Optional

from fastapi import FastAPI, HTTPException

from agent_hypervisor_amd.parallel.sharded import ShardedHypervisor
from hypervisor import __version__
from hypervisor.api.models import (
    AddStepRequest,
    AddStepResponse,
    AgentRingResponse,
    CreateSagaResponse,
    CreateSessionRequest,
    CreateSessionResponse,
    CreateVouchRequest,
    EventResponse,
    EventStatsResponse,
    ExecuteStepResponse,
    JoinSessionRequest,
    JoinSessionResponse,
    LiabilityExposureResponse,
    RingCheckRequest,
    RingCheckResponse,
    RingDistributionResponse,
    SagaDetailResponse,
    SessionDetailResponse,
    SessionListItem,
    StatsResponse,
    VouchResponse,
)
from hypervisor.models import ActionDescriptor, ExecutionRing
from hypervisor.saga.state_machine import SagaStateError


def create_sharded_app(shv: ShardedHypervisor) -> FastAPI:
    from contextlib import asynccontextmanager

    @asynccontextmanager
    async def lifespan(application: FastAPI):
        if shv._stopped is None:  # the RPC endpoint lives on the serving event loop
            await shv.start()
        yield
        await shv.shutdown()
        await shv.close()

    app = FastAPI(title="Agent Hypervisor (sharded)", version=__version__, lifespan=lifespan)

    async def call(coro, not_found=(ValueError, KeyError, SagaStateError)):
        try:
            return await coro
        except not_found as e:
            raise HTTPException(status_code=404, detail=str(e)) from e
        except HTTPException:
            raise
        except Exception as e:  # noqa: BLE001
            raise HTTPException(status_code=400, detail=str(e)) from e

    @app.get("/health")
    async def health() -> dict[str, Any]:
        return {"status": "ok", "version": __version__, "world": shv.world, "rank": shv.rank}

    @app.get("/api/v1/stats", response_model=StatsResponse)
    async def stats() -> StatsResponse:
        st = await call(shv.stats())
        ev = await call(shv.event_stats())
        return StatsResponse(version=__version__, event_count=ev["total_events"],
                             batched_sessions=shv.local.batched_sessions,
                             **{k: st[k] for k in ("total_sessions", "active_sessions", "total_participants",
                                                   "active_sagas", "total_vouches")})

    # ---------------------------------------------------------------- sessions
    @app.post("/api/v1/sessions", status_code=201, response_model=CreateSessionResponse)
    async def create_session(req: CreateSessionRequest) -> CreateSessionResponse:
        return CreateSessionResponse(**await call(shv.create_session(req.to_config(), req.creator_did, detail=True)))

    @app.get("/api/v1/sessions", response_model=list[SessionListItem])
    async def list_sessions(state: Optional[str] = None) -> list[SessionListItem]:
        return [SessionListItem(**{k: v for k, v in d.items() if k != "rank"})
                for d in await call(shv.list_sessions(state))]

    @app.get("/api/v1/sessions/{session_id}", response_model=SessionDetailResponse)
    async def get_session(session_id: str) -> SessionDetailResponse:
        return SessionDetailResponse(**await call(shv.get_session(session_id, detail=True)))

    @app.post("/api/v1/sessions/{session_id}/join", response_model=JoinSessionResponse)
    async def join(session_id: str, req: JoinSessionRequest) -> JoinSessionResponse:
        acts = [ActionDescriptor(**a) for a in req.actions] if req.actions else None
        ring = await call(shv.join_session(session_id, req.agent_did, sigma_raw=req.sigma_raw, actions=acts))
        ring = ExecutionRing(ring)
        return JoinSessionResponse(agent_did=req.agent_did, session_id=session_id, assigned_ring=ring.value,
                                   ring_name=ring.name)

    @app.post("/api/v1/sessions/{session_id}/activate")
    async def activate(session_id: str) -> dict[str, Any]:
        await call(shv.activate_session(session_id))
        return {"session_id": session_id, "state": "active"}

    @app.post("/api/v1/sessions/{session_id}/terminate")
    async def terminate(session_id: str) -> dict[str, Any]:
        root = await call(shv.terminate_session(session_id))
        return {"session_id": session_id, "state": "archived", "merkle_root": root}

    # ------------------------------------------------------------------- rings
    @app.get("/api/v1/sessions/{session_id}/rings", response_model=RingDistributionResponse)
    async def rings(session_id: str) -> RingDistributionResponse:
        return RingDistributionResponse(session_id=session_id,
                                        distribution=await call(shv.ring_distribution(session_id)))

    @app.get("/api/v1/agents/{agent_did}/ring", response_model=AgentRingResponse)
    async def agent_ring(agent_did: str) -> AgentRingResponse:
        r = await call(shv.agent_ring(agent_did))
        if r is None:
            raise HTTPException(status_code=404, detail=f"Agent {agent_did} not found in any session")
        return AgentRingResponse(agent_did=agent_did, ring=r["ring"], ring_name=ExecutionRing(r["ring"]).name,
                                 session_id=r["session_id"])

    @app.post("/api/v1/rings/check", response_model=RingCheckResponse)
    async def check_ring(req: RingCheckRequest) -> RingCheckResponse:
        return RingCheckResponse(**shv.check_ring(req.agent_ring, req.action, req.sigma_eff, req.has_consensus,
                                                  req.has_sre_witness))

    # ------------------------------------------------------------------- sagas
    @app.post("/api/v1/sessions/{session_id}/sagas", status_code=201, response_model=CreateSagaResponse)
    async def create_saga(session_id: str) -> CreateSagaResponse:
        return CreateSagaResponse(**await call(shv.create_saga(session_id, emit=True)))

    @app.get("/api/v1/sessions/{session_id}/sagas", response_model=list[SagaDetailResponse])
    async def list_sagas(session_id: str) -> list[SagaDetailResponse]:
        return [SagaDetailResponse(**d) for d in await call(shv.list_sagas(session_id))]

    @app.get("/api/v1/sagas/{saga_id}", response_model=SagaDetailResponse)
    async def get_saga(saga_id: str) -> SagaDetailResponse:
        return SagaDetailResponse(**await call(shv.get_saga(saga_id, detail=True)))

    @app.post("/api/v1/sagas/{saga_id}/steps", status_code=201, response_model=AddStepResponse)
    async def add_step(saga_id: str, req: AddStepRequest) -> AddStepResponse:
        return AddStepResponse(**await call(shv.add_step(saga_id, req.action_id, req.agent_did, req.execute_api,
                                                         req.undo_api, req.timeout_seconds, req.max_retries,
                                                         detail=True)))

    @app.post("/api/v1/sagas/{saga_id}/steps/{step_id}/execute", response_model=ExecuteStepResponse)
    async def execute(saga_id: str, step_id: str) -> ExecuteStepResponse:
        r = await call(shv.execute_step(saga_id, step_id, "api", rest=True))
        return ExecuteStepResponse(step_id=step_id, saga_id=saga_id, state=r["state"], error=r["error"])

    # --------------------------------------------------------------- liability
    @app.post("/api/v1/sessions/{session_id}/vouch", status_code=201, response_model=VouchResponse)
    async def vouch(session_id: str, req: CreateVouchRequest) -> VouchResponse:
        await call(shv.get_session(session_id))  # unknown session: 404 (the single-rank route's check)
        d = await call(shv.vouch(req.voucher_did, req.vouchee_did, session_id, req.voucher_sigma, req.bond_pct,
                                 None, emit=True), not_found=())
        return VouchResponse(**{k: d[k] for k in VouchResponse.model_fields})

    @app.get("/api/v1/sessions/{session_id}/vouches", response_model=list[VouchResponse])
    async def list_vouches(session_id: str) -> list[VouchResponse]:
        return [VouchResponse(**d) for d in await call(shv.list_vouches(session_id))]

    @app.get("/api/v1/agents/{agent_did}/liability", response_model=LiabilityExposureResponse)
    async def liability(agent_did: str) -> LiabilityExposureResponse:
        r = await call(shv.agent_liability(agent_did))
        pick = lambda d: VouchResponse(**{k: d[k] for k in VouchResponse.model_fields})  # noqa: E731
        return LiabilityExposureResponse(agent_did=agent_did, vouches_given=[pick(d) for d in r["vouches_given"]],
                                         vouches_received=[pick(d) for d in r["vouches_received"]],
                                         total_exposure=r["total_exposure"])

    # ------------------------------------------------------------------ events
    @app.get("/api/v1/events", response_model=list[EventResponse])
    async def events(event_type: Optional[str] = None, session_id: Optional[str] = None,
                     agent_did: Optional[str] = None, limit: Optional[int] = None) -> list[EventResponse]:
        if event_type:
            from hypervisor.observability.event_bus import EventType

            try:
                EventType(event_type)
            except ValueError as e:
                raise HTTPException(status_code=400, detail=f"Unknown event type: {event_type}") from e
        return [EventResponse(**d) for d in await call(shv.events(event_type, session_id, agent_did, limit))]

    @app.get("/api/v1/events/stats", response_model=EventStatsResponse)
    async def event_stats() -> EventStatsResponse:
        return EventStatsResponse(**await call(shv.event_stats()))

    return app
