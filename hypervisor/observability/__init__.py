"""Observability: structured event bus and causal trace ids."""

from hypervisor.observability.causal_trace import CausalTraceId
from hypervisor.observability.event_bus import EventType, HypervisorEvent, HypervisorEventBus

__all__ = ["EventType", "HypervisorEvent", "HypervisorEventBus", "CausalTraceId"]
