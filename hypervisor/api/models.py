"""Wire schemas of the REST front-end.

Field names and defaults are the public contract of the reference API
(reference api/models.py:15-245, 22 models); the request models convert
themselves into core objects so the route handlers stay thin.
"""

from __future__ import annotations

from typing import Any, Optional

from pydantic import BaseModel, Field

from hypervisor.models import ConsistencyMode, SessionConfig


def _iso(t) -> Optional[str]:
    return t.isoformat() if t is not None else None


# ------------------------------------------------------------------ sessions


class CreateSessionRequest(BaseModel):
    creator_did: str = Field(..., description="DID of the session creator")
    consistency_mode: ConsistencyMode = ConsistencyMode.EVENTUAL
    max_participants: int = 10
    max_duration_seconds: int = 3600
    min_sigma_eff: float = 0.60
    enable_audit: bool = True
    enable_blockchain_commitment: bool = False

    def to_config(self) -> SessionConfig:
        return SessionConfig(**self.model_dump(exclude={"creator_did"}))


class ParticipantInfo(BaseModel):
    agent_did: str
    ring: int
    sigma_raw: float
    sigma_eff: float
    joined_at: str
    is_active: bool

    @classmethod
    def of(cls, p) -> "ParticipantInfo":
        return cls(agent_did=p.agent_did, ring=p.ring.value, sigma_raw=p.sigma_raw, sigma_eff=p.sigma_eff,
                   joined_at=p.joined_at.isoformat(), is_active=p.is_active)


class CreateSessionResponse(BaseModel):
    session_id: str
    state: str
    consistency_mode: str
    created_at: str


class SessionListItem(BaseModel):
    session_id: str
    state: str
    consistency_mode: str
    participant_count: int
    created_at: str

    @classmethod
    def of(cls, sso) -> "SessionListItem":
        return cls(session_id=sso.session_id, state=sso.state.value, consistency_mode=sso.consistency_mode.value,
                   participant_count=sso.participant_count, created_at=sso.created_at.isoformat())


class SessionDetailResponse(BaseModel):
    session_id: str
    state: str
    consistency_mode: str
    creator_did: str
    participant_count: int
    participants: list[ParticipantInfo]
    created_at: str
    terminated_at: Optional[str] = None
    sagas: list[dict[str, Any]] = []


class JoinSessionRequest(BaseModel):
    agent_did: str = Field(..., description="DID of the joining agent")
    actions: Optional[list[dict[str, Any]]] = None
    sigma_raw: float = 0.0


class JoinSessionResponse(BaseModel):
    agent_did: str
    session_id: str
    assigned_ring: int
    ring_name: str


# --------------------------------------------------------------------- rings


class RingDistributionResponse(BaseModel):
    session_id: str
    distribution: dict[str, list[str]]


class AgentRingResponse(BaseModel):
    agent_did: str
    ring: int
    ring_name: str
    session_id: str


class RingCheckRequest(BaseModel):
    agent_ring: int = Field(..., description="Agent's current ring level (0-3)")
    action: dict[str, Any] = Field(..., description="ActionDescriptor fields")
    sigma_eff: float = Field(..., description="Agent's effective reputation score")
    has_consensus: bool = False
    has_sre_witness: bool = False


class RingCheckResponse(BaseModel):
    allowed: bool
    required_ring: int
    agent_ring: int
    sigma_eff: float
    reason: str
    requires_consensus: bool = False
    requires_sre_witness: bool = False


# --------------------------------------------------------------------- sagas


class CreateSagaResponse(BaseModel):
    saga_id: str
    session_id: str
    state: str
    created_at: str


class SagaDetailResponse(BaseModel):
    saga_id: str
    session_id: str
    state: str
    created_at: str
    completed_at: Optional[str] = None
    error: Optional[str] = None
    steps: list[dict[str, Any]]

    @classmethod
    def of(cls, saga) -> "SagaDetailResponse":
        steps = [
            {"step_id": s.step_id, "action_id": s.action_id, "agent_did": s.agent_did, "state": s.state.value,
             "error": s.error}
            for s in saga.steps
        ]
        return cls(saga_id=saga.saga_id, session_id=saga.session_id, state=saga.state.value,
                   created_at=saga.created_at.isoformat(), completed_at=_iso(saga.completed_at), error=saga.error,
                   steps=steps)


class AddStepRequest(BaseModel):
    action_id: str
    agent_did: str
    execute_api: str
    undo_api: Optional[str] = None
    timeout_seconds: int = 300
    max_retries: int = 0


class AddStepResponse(BaseModel):
    step_id: str
    saga_id: str
    action_id: str
    state: str


class ExecuteStepResponse(BaseModel):
    step_id: str
    saga_id: str
    state: str
    error: Optional[str] = None


# ----------------------------------------------------------------- liability


class CreateVouchRequest(BaseModel):
    voucher_did: str = Field(..., description="DID of the vouching agent")
    vouchee_did: str = Field(..., description="DID of the agent being vouched for")
    voucher_sigma: float = Field(..., description="Voucher's raw reputation score")
    bond_pct: Optional[float] = None
    expiry: Optional[str] = None


class VouchResponse(BaseModel):
    vouch_id: str
    voucher_did: str
    vouchee_did: str
    session_id: str
    bonded_amount: float
    bonded_sigma_pct: float
    is_active: bool

    @classmethod
    def of(cls, v) -> "VouchResponse":
        return cls(vouch_id=v.vouch_id, voucher_did=v.voucher_did, vouchee_did=v.vouchee_did,
                   session_id=v.session_id, bonded_amount=v.bonded_amount, bonded_sigma_pct=v.bonded_sigma_pct,
                   is_active=v.is_active)


class LiabilityExposureResponse(BaseModel):
    agent_did: str
    vouches_given: list[VouchResponse]
    vouches_received: list[VouchResponse]
    total_exposure: float


# -------------------------------------------------------------------- events


class EventResponse(BaseModel):
    event_id: str
    event_type: str
    timestamp: str
    session_id: Optional[str] = None
    agent_did: Optional[str] = None
    causal_trace_id: Optional[str] = None
    payload: dict[str, Any] = {}

    @classmethod
    def of(cls, e) -> "EventResponse":
        return cls(event_id=e.event_id, event_type=e.event_type.value, timestamp=e.timestamp.isoformat(),
                   session_id=e.session_id, agent_did=e.agent_did, causal_trace_id=e.causal_trace_id,
                   payload=e.payload)


class EventStatsResponse(BaseModel):
    total_events: int
    by_type: dict[str, int]


class StatsResponse(BaseModel):
    version: str
    total_sessions: int
    active_sessions: int
    total_participants: int
    active_sagas: int
    total_vouches: int
    event_count: int
    batched_sessions: int = 0  # sessions run by the batched device pipeline (readable by id)


# ------------------------------------------------- MI355X batch extension


class PipelineBatchRequest(BaseModel):
    """Run the full governance pipeline for many synthetic sessions on the
    device engine (create → join → activate → saga step → audit → terminate)."""

    sessions: int = Field(1024, ge=1, le=1 << 20)
    deltas: int = Field(3, ge=0, le=8)
    seed: int = 0


class PipelineBatchResponse(BaseModel):
    sessions: int
    completed: int
    device: str
    elapsed_ms: float
    sessions_per_second: float
    sample_merkle_root: Optional[str] = None
    sample_session_id: Optional[str] = None
