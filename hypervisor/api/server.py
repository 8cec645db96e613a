"""REST front-end of the hypervisor (FastAPI).

Same routes, status codes and payloads as the reference server
(reference api/server.py:138-645: ``/health`` plus 20 ``/api/v1`` routes; error
mapping ValueError → 404, other failures → 400, unknown event type → 400), with
these differences:

* state lives on ``app.state.hv`` (an :class:`ApiState`), created by
  :func:`create_app` and re-created by the lifespan, instead of module globals —
  several apps can coexist (tests, multi-tenant serving);
* the event bus is wired into the :class:`Hypervisor`, so ``/api/v1/events``
  reports lifecycle events (the reference's bus is never fed and always
  returns ``[]``);
* handlers use public query methods (``Hypervisor.sessions``, ``find_saga``,
  ``VouchingEngine.records``) instead of private dicts;
* ``POST /api/v1/engine/pipeline`` exposes the batched MI355X governance engine
  (:class:`agent_hypervisor_amd.models.engine.GovernanceEngine`).
"""

from __future__ import annotations

import time
from contextlib import asynccontextmanager
from dataclasses import dataclass, field
from typing import Any, Optional

from fastapi import APIRouter, FastAPI, HTTPException, Query, Request
from fastapi.middleware.cors import CORSMiddleware

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
    ParticipantInfo,
    PipelineBatchRequest,
    PipelineBatchResponse,
    RingCheckRequest,
    RingCheckResponse,
    RingDistributionResponse,
    SagaDetailResponse,
    SessionDetailResponse,
    SessionListItem,
    StatsResponse,
    VouchResponse,
)
from hypervisor.core import Hypervisor
from hypervisor.models import ActionDescriptor, ExecutionRing
from hypervisor.observability.event_bus import EventType, HypervisorEventBus


@dataclass
class ApiState:
    bus: HypervisorEventBus = field(default_factory=HypervisorEventBus)
    hv: Optional[Hypervisor] = None

    def __post_init__(self) -> None:
        if self.hv is None:
            self.hv = Hypervisor(event_bus=self.bus)
        elif self.hv.event_bus is None:
            self.hv.event_bus = self.bus


def _state(request: Request) -> ApiState:
    st = getattr(request.app.state, "hv", None)
    if st is None:
        raise HTTPException(status_code=503, detail="Hypervisor not initialized")
    return st


def _managed(st: ApiState, session_id: str):
    m = st.hv.get_session(session_id)
    if m is None:
        raise HTTPException(status_code=404, detail=f"Session {session_id} not found")
    return m


async def _guard(coro):
    """Await a core call with the reference's error mapping."""
    try:
        return await coro
    except HTTPException:
        raise
    except ValueError as e:
        raise HTTPException(status_code=404, detail=str(e)) from e
    except Exception as e:  # noqa: BLE001 - surfaced as a 400 like the reference
        raise HTTPException(status_code=400, detail=str(e)) from e


router = APIRouter()

# ------------------------------------------------------------------ health


@router.get("/health", tags=["Health"])
async def health_check() -> dict[str, str]:
    return {"status": "ok", "version": __version__}


@router.get("/api/v1/stats", response_model=StatsResponse, tags=["Health"])
async def get_stats(request: Request) -> StatsResponse:
    st = _state(request)
    hv = st.hv
    c = hv.counters()  # device-backed: one reduction over the rows, no per-session snapshot
    return StatsResponse(
        version=__version__,
        total_sessions=c["total_sessions"],
        active_sessions=c["active_sessions"],
        total_participants=c["total_participants"],
        active_sagas=c["active_sagas"],
        total_vouches=c["total_vouches"],
        event_count=st.bus.event_count,
        batched_sessions=hv.batched_sessions,
    )


# ---------------------------------------------------------------- sessions


@router.post("/api/v1/sessions", response_model=CreateSessionResponse, status_code=201, tags=["Sessions"])
async def create_session(req: CreateSessionRequest, request: Request) -> CreateSessionResponse:
    m = await _state(request).hv.create_session(config=req.to_config(), creator_did=req.creator_did)
    sso = m.sso
    return CreateSessionResponse(session_id=sso.session_id, state=sso.state.value,
                                 consistency_mode=sso.consistency_mode.value, created_at=sso.created_at.isoformat())


@router.get("/api/v1/sessions", response_model=list[SessionListItem], tags=["Sessions"])
async def list_sessions(
    request: Request, state: Optional[str] = Query(None, description="Filter by session state")
) -> list[SessionListItem]:
    return [SessionListItem.of(x) for x in _state(request).hv.snapshots() if not state or x.state.value == state]


@router.get("/api/v1/sessions/{session_id}", response_model=SessionDetailResponse, tags=["Sessions"])
async def get_session(session_id: str, request: Request) -> SessionDetailResponse:
    m = _managed(_state(request), session_id)
    sso = m.sso
    return SessionDetailResponse(
        session_id=sso.session_id,
        state=sso.state.value,
        consistency_mode=sso.consistency_mode.value,
        creator_did=sso.creator_did,
        participant_count=sso.participant_count,
        participants=[ParticipantInfo.of(p) for p in sso.participants],
        created_at=sso.created_at.isoformat(),
        terminated_at=sso.terminated_at.isoformat() if sso.terminated_at else None,
        sagas=[s.to_dict() for s in m.saga.sagas],
    )


@router.post("/api/v1/sessions/{session_id}/join", response_model=JoinSessionResponse, tags=["Sessions"])
async def join_session(session_id: str, req: JoinSessionRequest, request: Request) -> JoinSessionResponse:
    hv = _state(request).hv

    async def run():
        actions = [ActionDescriptor(**a) for a in req.actions] if req.actions else None
        return await hv.join_session(session_id=session_id, agent_did=req.agent_did, actions=actions,
                                     sigma_raw=req.sigma_raw)

    ring = await _guard(run())
    return JoinSessionResponse(agent_did=req.agent_did, session_id=session_id, assigned_ring=ring.value,
                               ring_name=ring.name)


@router.post("/api/v1/sessions/{session_id}/activate", tags=["Sessions"])
async def activate_session(session_id: str, request: Request) -> dict[str, str]:
    await _guard(_state(request).hv.activate_session(session_id))
    return {"session_id": session_id, "state": "active"}


@router.post("/api/v1/sessions/{session_id}/terminate", tags=["Sessions"])
async def terminate_session(session_id: str, request: Request) -> dict[str, Any]:
    root = await _guard(_state(request).hv.terminate_session(session_id))
    return {"session_id": session_id, "state": "archived", "merkle_root": root}


# ------------------------------------------------------------------- rings


@router.get("/api/v1/sessions/{session_id}/rings", response_model=RingDistributionResponse, tags=["Rings"])
async def get_ring_distribution(session_id: str, request: Request) -> RingDistributionResponse:
    dist: dict[str, list[str]] = {}
    for p in _managed(_state(request), session_id).sso.participants:
        dist.setdefault(p.ring.name, []).append(p.agent_did)
    return RingDistributionResponse(session_id=session_id, distribution=dist)


@router.get("/api/v1/agents/{agent_did}/ring", response_model=AgentRingResponse, tags=["Rings"])
async def get_agent_ring(agent_did: str, request: Request) -> AgentRingResponse:
    for x in _state(request).hv.snapshots(parts=True):
        for p in x.participants:
            if p.agent_did == agent_did and p.is_active:
                return AgentRingResponse(agent_did=agent_did, ring=p.ring.value, ring_name=p.ring.name,
                                         session_id=x.session_id)
    raise HTTPException(status_code=404, detail=f"Agent {agent_did} not found in any session")


@router.post("/api/v1/rings/check", response_model=RingCheckResponse, tags=["Rings"])
async def check_ring_access(req: RingCheckRequest, request: Request) -> RingCheckResponse:
    hv = _state(request).hv
    r = hv.ring_enforcer.check(
        agent_ring=ExecutionRing(req.agent_ring),
        action=ActionDescriptor(**req.action),
        sigma_eff=req.sigma_eff,
        has_consensus=req.has_consensus,
        has_sre_witness=req.has_sre_witness,
    )
    return RingCheckResponse(allowed=r.allowed, required_ring=r.required_ring.value, agent_ring=r.agent_ring.value,
                             sigma_eff=r.sigma_eff, reason=r.reason, requires_consensus=r.requires_consensus,
                             requires_sre_witness=r.requires_sre_witness)


# ------------------------------------------------------------------- sagas


@router.post("/api/v1/sessions/{session_id}/sagas", response_model=CreateSagaResponse, status_code=201,
             tags=["Sagas"])
async def create_saga(session_id: str, request: Request) -> CreateSagaResponse:
    st = _state(request)
    saga = _managed(st, session_id).saga.create_saga(session_id)
    st.hv._emit(EventType.SAGA_CREATED, session_id, saga_id=saga.saga_id)
    return CreateSagaResponse(saga_id=saga.saga_id, session_id=saga.session_id, state=saga.state.value,
                              created_at=saga.created_at.isoformat())


@router.get("/api/v1/sessions/{session_id}/sagas", response_model=list[SagaDetailResponse], tags=["Sagas"])
async def list_sagas(session_id: str, request: Request) -> list[SagaDetailResponse]:
    return [SagaDetailResponse.of(s) for s in _managed(_state(request), session_id).saga.sagas]


def _find_saga(request: Request, saga_id: str, detail: Optional[str] = None):
    m, saga = _state(request).hv.find_saga(saga_id)
    if saga is None:
        raise HTTPException(status_code=404, detail=detail or f"Saga {saga_id} not found")
    return m, saga


@router.get("/api/v1/sagas/{saga_id}", response_model=SagaDetailResponse, tags=["Sagas"])
async def get_saga(saga_id: str, request: Request) -> SagaDetailResponse:
    return SagaDetailResponse.of(_find_saga(request, saga_id)[1])


@router.post("/api/v1/sagas/{saga_id}/steps", response_model=AddStepResponse, status_code=201, tags=["Sagas"])
async def add_saga_step(saga_id: str, req: AddStepRequest, request: Request) -> AddStepResponse:
    m, _ = _find_saga(request, saga_id)
    try:
        step = m.saga.add_step(saga_id=saga_id, **req.model_dump())
    except Exception as e:  # noqa: BLE001
        raise HTTPException(status_code=400, detail=str(e)) from e
    return AddStepResponse(step_id=step.step_id, saga_id=saga_id, action_id=step.action_id, state=step.state.value)


async def _api_executor() -> dict[str, str]:
    return {"status": "executed_via_api"}


@router.post("/api/v1/sagas/{saga_id}/steps/{step_id}/execute", response_model=ExecuteStepResponse,
             tags=["Sagas"])
async def execute_saga_step(saga_id: str, step_id: str, request: Request) -> ExecuteStepResponse:
    missing = f"Saga {saga_id} or step {step_id} not found"
    m, saga = _find_saga(request, saga_id, missing)
    try:
        await m.saga.execute_step(saga_id, step_id, _api_executor)
    except Exception as e:  # noqa: BLE001
        raise HTTPException(status_code=400, detail=str(e)) from e
    for s in saga.steps:
        if s.step_id == step_id:
            et = EventType.SAGA_STEP_COMMITTED if s.state.value == "committed" else EventType.SAGA_STEP_FAILED
            _state(request).hv._emit(et, saga.session_id, s.agent_did, saga_id=saga_id, step_id=step_id)
            return ExecuteStepResponse(step_id=step_id, saga_id=saga_id, state=s.state.value, error=s.error)
    raise HTTPException(status_code=404, detail=missing)


# --------------------------------------------------------------- liability


@router.post("/api/v1/sessions/{session_id}/vouch", response_model=VouchResponse, status_code=201,
             tags=["Liability"])
async def create_vouch(session_id: str, req: CreateVouchRequest, request: Request) -> VouchResponse:
    st = _state(request)
    _managed(st, session_id)
    try:
        rec = st.hv.vouching.vouch(voucher_did=req.voucher_did, vouchee_did=req.vouchee_did, session_id=session_id,
                                   voucher_sigma=req.voucher_sigma, bond_pct=req.bond_pct)
    except Exception as e:  # noqa: BLE001
        raise HTTPException(status_code=400, detail=str(e)) from e
    st.hv._emit(EventType.VOUCH_CREATED, session_id, req.voucher_did, vouch_id=rec.vouch_id,
                vouchee_did=req.vouchee_did, bonded_amount=rec.bonded_amount)
    return VouchResponse.of(rec)


@router.get("/api/v1/sessions/{session_id}/vouches", response_model=list[VouchResponse], tags=["Liability"])
async def list_vouches(session_id: str, request: Request) -> list[VouchResponse]:
    st = _state(request)
    _managed(st, session_id)
    return [VouchResponse.of(v) for v in st.hv.vouching.records(session_id)]


@router.get("/api/v1/agents/{agent_did}/liability", response_model=LiabilityExposureResponse, tags=["Liability"])
async def get_agent_liability(agent_did: str, request: Request) -> LiabilityExposureResponse:
    given, received, exposure = [], [], 0.0
    for v in _state(request).hv.vouching.records():
        if v.voucher_did == agent_did:
            given.append(VouchResponse.of(v))
            if v.is_active and not v.is_expired:
                exposure += v.bonded_amount
        if v.vouchee_did == agent_did:
            received.append(VouchResponse.of(v))
    return LiabilityExposureResponse(agent_did=agent_did, vouches_given=given, vouches_received=received,
                                     total_exposure=exposure)


# ------------------------------------------------------------------ events


@router.get("/api/v1/events", response_model=list[EventResponse], tags=["Events"])
async def query_events(
    request: Request,
    event_type: Optional[str] = Query(None, description="Filter by event type"),
    session_id: Optional[str] = Query(None, description="Filter by session ID"),
    agent_did: Optional[str] = Query(None, description="Filter by agent DID"),
    limit: Optional[int] = Query(None, description="Max events to return"),
) -> list[EventResponse]:
    et = None
    if event_type:
        try:
            et = EventType(event_type)
        except ValueError as e:
            raise HTTPException(status_code=400, detail=f"Unknown event type: {event_type}") from e
    events = _state(request).bus.query(event_type=et, session_id=session_id, agent_did=agent_did, limit=limit)
    return [EventResponse.of(e) for e in events]


@router.get("/api/v1/events/stats", response_model=EventStatsResponse, tags=["Events"])
async def get_event_stats(request: Request) -> EventStatsResponse:
    bus = _state(request).bus
    return EventStatsResponse(total_events=bus.event_count, by_type=bus.type_counts())


# ------------------------------------------------------------- audit


@router.get("/api/v1/audit/verify", tags=["Audit"])
async def verify_audit(
    request: Request,
    session_id: Optional[list[str]] = Query(None, description="Sessions to audit (default: all)"),
    device: Optional[str] = Query(None, description="cuda | cpu (default: GPU for large batches)"),
) -> dict[str, Any]:
    """Batched audit: delta chains (K10), committed roots (K09), VFS contents (K11)."""
    hv = _state(request).hv
    try:
        return hv.verify_audit(session_id, device=device).to_dict()
    except ValueError as e:
        raise HTTPException(status_code=404, detail=str(e)) from e


# ------------------------------------------------- MI355X batched engine


@router.post("/api/v1/engine/pipeline", response_model=PipelineBatchResponse, tags=["Engine"])
async def run_pipeline_batch(req: PipelineBatchRequest, request: Request) -> PipelineBatchResponse:
    hv = _state(request).hv
    try:
        t0 = time.perf_counter()
        run = hv.pipeline_batch(req.sessions, deltas=req.deltas)
        dt = time.perf_counter() - t0
    except Exception as e:  # noqa: BLE001
        raise HTTPException(status_code=400, detail=str(e)) from e
    sid = run.session_ids[0] if req.sessions > 0 else None
    return PipelineBatchResponse(
        sessions=req.sessions,
        completed=run.ok,
        device=str(hv._store.device),
        elapsed_ms=dt * 1e3,
        sessions_per_second=req.sessions / dt if dt > 0 else 0.0,
        sample_merkle_root=run.roots.get(sid) if sid is not None else None,
        sample_session_id=sid,
    )


# --------------------------------------------------------------- factory


def create_app(hypervisor: Optional[Hypervisor] = None, event_bus: Optional[HypervisorEventBus] = None) -> FastAPI:
    """Build the FastAPI application (optionally around an existing hypervisor)."""

    @asynccontextmanager
    async def lifespan(application: FastAPI):
        if getattr(application.state, "hv", None) is None:
            application.state.hv = ApiState(bus=event_bus or HypervisorEventBus(), hv=hypervisor)
        from hypervisor.config import tune_gc

        tune_gc()  # a serving process: collector thresholds for many in-flight sessions
        yield
        application.state.hv = None

    application = FastAPI(
        title="Agent Hypervisor API",
        description=(
            "REST API of the MI355X agent hypervisor: shared sessions, execution rings, joint liability, "
            "saga orchestration and Merkle-chained audit, plus the batched device engine."
        ),
        version=__version__,
        lifespan=lifespan,
    )
    application.add_middleware(CORSMiddleware, allow_origins=["*"], allow_credentials=True, allow_methods=["*"],
                               allow_headers=["*"])
    application.state.hv = ApiState(bus=event_bus or HypervisorEventBus(), hv=hypervisor)
    application.include_router(router)
    from hypervisor.api.dashboard import router as dashboard_router

    application.include_router(dashboard_router)
    return application


app = create_app()
