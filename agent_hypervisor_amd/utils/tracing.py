"""Host-stage tracing: roctx ranges + an in-process span log.

Disabled by default (one boolean check per call).  With ``AHV_TRACE=1`` or
:func:`set_tracing(True)`:

* every :func:`span` / :func:`traced` region is pushed as a roctx range (via
  torch's ROCm tracer hooks), so ``rocprofv3 --marker-trace`` shows the host
  stages (create/join/activate/terminate, engine launches, graph replays)
  aligned with the kernels they launch;
* spans are also kept in memory with wall-clock durations: :func:`summary`
  gives per-stage counts / total / p50 (the reference's §3.3 stage breakdown,
  measurable on any box) and :func:`export_chrome_trace` writes a
  chrome://tracing / Perfetto JSON file.
"""

from __future__ import annotations

import functools
import inspect
import json
import os
import statistics
import threading
import time
from contextlib import contextmanager
from typing import Optional

_enabled = os.environ.get("AHV_TRACE", "0").strip().lower() in ("1", "true", "yes", "on")
_spans: list[tuple[str, int, int, int, dict]] = []
_lock = threading.Lock()
_MAX_SPANS = 1_000_000


def set_tracing(on: bool) -> None:
    """Enable/disable tracing.  Enabling also instruments the host stages
    (Hypervisor lifecycle, saga orchestrator, device engines); disabling
    restores the original methods, so an untraced process pays nothing."""
    global _enabled
    _enabled = bool(on)
    if _enabled:
        instrument()
    else:
        uninstrument()


# (module, class, method, span name) of the instrumented host stages
_STAGES = (
    ("hypervisor.core", "Hypervisor", "create_session", "hypervisor.create_session"),
    ("hypervisor.core", "Hypervisor", "join_session", "hypervisor.join_session"),
    ("hypervisor.core", "Hypervisor", "activate_session", "hypervisor.activate_session"),
    ("hypervisor.core", "Hypervisor", "terminate_session", "hypervisor.terminate_session"),
    ("hypervisor.core", "Hypervisor", "verify_behavior", "hypervisor.verify_behavior"),
    ("hypervisor.saga.orchestrator", "SagaOrchestrator", "execute_step", "saga.execute_step"),
    ("hypervisor.saga.orchestrator", "SagaOrchestrator", "compensate", "saga.compensate"),
    ("hypervisor._device", "DeviceSagaOrchestrator", "execute_step", "saga.execute_step"),
    ("hypervisor._device", "DeviceSagaOrchestrator", "compensate", "saga.compensate"),
    ("hypervisor._device", "DeviceDeltaEngine", "capture", "audit.capture"),
    ("hypervisor._device", "DeviceDeltaEngine", "verify_chain", "audit.verify_chain"),
    ("hypervisor._device", "DeviceSlashingEngine", "slash", "liability.slash"),
    ("agent_hypervisor_amd.models.engine", "GovernanceEngine", "run_pipeline", "engine.run_pipeline"),
    ("agent_hypervisor_amd.models.saga_engine", "SagaBatchEngine", "run", "saga_engine.run"),
    ("agent_hypervisor_amd.models.saga_engine", "SagaBatchEngine", "run_step_loop", "saga_engine.run_step_loop"),
    ("agent_hypervisor_amd.runtime.graphs", "PipelineGraph", "step", "graph.step"),
)
_originals: dict[tuple[str, str, str], object] = {}


def instrument() -> None:
    import importlib

    for mod, cls, meth, label in _STAGES:
        key = (mod, cls, meth)
        if key in _originals:
            continue
        klass = getattr(importlib.import_module(mod), cls)
        orig = klass.__dict__[meth]
        _originals[key] = orig
        setattr(klass, meth, traced(label)(orig))


def uninstrument() -> None:
    import importlib

    for (mod, cls, meth), orig in list(_originals.items()):
        setattr(getattr(importlib.import_module(mod), cls), meth, orig)
        del _originals[(mod, cls, meth)]


def enabled() -> bool:
    return _enabled


def _roctx():
    try:
        import torch

        if torch.cuda.is_available():
            return torch.cuda.nvtx  # routed to roctx on ROCm builds
    except Exception:  # noqa: BLE001
        pass
    return None


@contextmanager
def span(name: str, **attrs):
    if not _enabled:
        yield
        return
    tx = _roctx()
    if tx is not None:
        tx.range_push(name)
    t0 = time.perf_counter_ns()
    try:
        yield
    finally:
        dt = time.perf_counter_ns() - t0
        if tx is not None:
            tx.range_pop()
        with _lock:
            if len(_spans) < _MAX_SPANS:
                _spans.append((name, t0, dt, threading.get_ident(), attrs))


def traced(name: Optional[str] = None):
    """Decorator: wrap a function or coroutine function in :func:`span`."""

    def deco(fn):
        label = name or fn.__qualname__
        if inspect.iscoroutinefunction(fn):

            @functools.wraps(fn)
            async def aw(*a, **k):
                if not _enabled:
                    return await fn(*a, **k)
                with span(label):
                    return await fn(*a, **k)

            return aw

        @functools.wraps(fn)
        def w(*a, **k):
            if not _enabled:
                return fn(*a, **k)
            with span(label):
                return fn(*a, **k)

        return w

    return deco


def spans() -> list[tuple[str, int, int, int, dict]]:
    with _lock:
        return list(_spans)


def clear() -> None:
    with _lock:
        _spans.clear()


def summary() -> dict[str, dict[str, float]]:
    """name → {count, total_us, mean_us, p50_us}."""
    by: dict[str, list[int]] = {}
    for name, _, dt, _, _ in spans():
        by.setdefault(name, []).append(dt)
    return {
        n: {"count": len(v), "total_us": sum(v) / 1e3, "mean_us": statistics.mean(v) / 1e3,
            "p50_us": statistics.median(v) / 1e3}
        for n, v in sorted(by.items())
    }


def export_chrome_trace(path: str) -> str:
    events = [
        {"name": n, "ph": "X", "ts": t0 / 1e3, "dur": dt / 1e3, "pid": os.getpid(), "tid": tid, "args": attrs}
        for n, t0, dt, tid, attrs in spans()
    ]
    with open(path, "w") as f:
        json.dump({"traceEvents": events, "displayTimeUnit": "ns"}, f)
    return path
