"""Agent Hypervisor — MI355X-native runtime supervisor for multi-agent shared sessions.

Same public API as ``imran-siddique/agent-hypervisor`` v2.0.0 (58 exports, same
module paths), rebuilt on a native core: the audit hash path runs on the shared
host/gfx950 SHA-256 engine, and the batched governance pipeline (σ_eff ring gate,
liability accounting, saga FSM, Merkle-chained audit) runs as hand-written CDNA4
HIP kernels over device-resident session tables, sharded across GPUs with RCCL
(see :mod:`agent_hypervisor_amd`).

    >>> from hypervisor import Hypervisor, SessionConfig
    >>> hv = Hypervisor()
    >>> s = await hv.create_session(SessionConfig(), creator_did="did:mesh:admin")
"""

__version__ = "2.0.0"

from hypervisor.models import (
    ConsistencyMode,
    ExecutionRing,
    ReversibilityLevel,
    SessionConfig,
    SessionState,
)
from hypervisor.session import SharedSessionObject
from hypervisor.session.sso import SessionVFS, VFSEdit, VFSPermissionError
from hypervisor.session.vector_clock import CausalViolationError, VectorClock, VectorClockManager
from hypervisor.session.intent_locks import DeadlockError, IntentLockManager, LockContentionError, LockIntent
from hypervisor.session.isolation import IsolationLevel
from hypervisor.liability.vouching import VouchingEngine, VouchRecord
from hypervisor.liability.slashing import SlashingEngine
from hypervisor.liability import LiabilityMatrix
from hypervisor.liability.attribution import AttributionResult, CausalAttributor
from hypervisor.liability.quarantine import QuarantineManager, QuarantineReason
from hypervisor.liability.ledger import LedgerEntryType, LiabilityLedger
from hypervisor.rings.enforcer import RingEnforcer
from hypervisor.rings.classifier import ActionClassifier
from hypervisor.rings.elevation import RingElevation, RingElevationManager
from hypervisor.rings.breach_detector import BreachSeverity, RingBreachDetector
from hypervisor.reversibility.registry import ReversibilityRegistry
from hypervisor.saga.orchestrator import SagaOrchestrator, SagaTimeoutError
from hypervisor.saga.state_machine import SagaState, StepState
from hypervisor.saga.fan_out import FanOutOrchestrator, FanOutPolicy
from hypervisor.saga.checkpoint import CheckpointManager, SemanticCheckpoint
from hypervisor.saga.dsl import SagaDefinition, SagaDSLParser
from hypervisor.audit.delta import DeltaEngine
from hypervisor.audit.commitment import CommitmentEngine
from hypervisor.audit.gc import EphemeralGC
from hypervisor.verification.history import TransactionHistoryVerifier
from hypervisor.observability.event_bus import EventType, HypervisorEvent, HypervisorEventBus
from hypervisor.observability.causal_trace import CausalTraceId
from hypervisor.security.rate_limiter import AgentRateLimiter, RateLimitExceeded
from hypervisor.security.kill_switch import KillResult, KillSwitch
from hypervisor.core import Hypervisor

__all__ = [
    "__version__",
    "Hypervisor",
    "ConsistencyMode",
    "ExecutionRing",
    "ReversibilityLevel",
    "SessionConfig",
    "SessionState",
    "SharedSessionObject",
    "SessionVFS",
    "VFSEdit",
    "VFSPermissionError",
    "VectorClock",
    "VectorClockManager",
    "CausalViolationError",
    "IntentLockManager",
    "LockIntent",
    "LockContentionError",
    "DeadlockError",
    "IsolationLevel",
    "VouchRecord",
    "VouchingEngine",
    "SlashingEngine",
    "LiabilityMatrix",
    "CausalAttributor",
    "AttributionResult",
    "QuarantineManager",
    "QuarantineReason",
    "LiabilityLedger",
    "LedgerEntryType",
    "RingEnforcer",
    "ActionClassifier",
    "RingElevationManager",
    "RingElevation",
    "RingBreachDetector",
    "BreachSeverity",
    "ReversibilityRegistry",
    "SagaOrchestrator",
    "SagaTimeoutError",
    "SagaState",
    "StepState",
    "FanOutOrchestrator",
    "FanOutPolicy",
    "CheckpointManager",
    "SemanticCheckpoint",
    "SagaDSLParser",
    "SagaDefinition",
    "DeltaEngine",
    "CommitmentEngine",
    "EphemeralGC",
    "TransactionHistoryVerifier",
    "HypervisorEventBus",
    "EventType",
    "HypervisorEvent",
    "CausalTraceId",
    "AgentRateLimiter",
    "RateLimitExceeded",
    "KillSwitch",
    "KillResult",
]

# AHV_TRACE=1: instrument the host stages with roctx ranges + span log (§5.1)
from agent_hypervisor_amd.utils import tracing as _tracing  # noqa: E402

if _tracing.enabled():
    _tracing.instrument()
