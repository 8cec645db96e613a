"""Saga: orchestration, fan-out, semantic checkpoints, declarative DSL."""

from hypervisor.saga.checkpoint import CheckpointManager, SemanticCheckpoint
from hypervisor.saga.dsl import SagaDefinition, SagaDSLError, SagaDSLParser
from hypervisor.saga.fan_out import FanOutGroup, FanOutOrchestrator, FanOutPolicy

__all__ = [
    "FanOutOrchestrator",
    "FanOutGroup",
    "FanOutPolicy",
    "CheckpointManager",
    "SemanticCheckpoint",
    "SagaDSLParser",
    "SagaDefinition",
    "SagaDSLError",
]
