"""Serving-process knobs: GC thresholds, the integer-µs clock, store telemetry."""

from __future__ import annotations

import gc

import pytest

from hypervisor import _clock
from hypervisor.config import RUNTIME, tune_gc


def test_tune_gc_sets_and_returns_previous(monkeypatch):
    before = gc.get_threshold()
    try:
        monkeypatch.setattr(RUNTIME, "gc_threshold", "12345,7,9")
        old = tune_gc()
        assert old == before and gc.get_threshold() == (12345, 7, 9)
        monkeypatch.setattr(RUNTIME, "gc_threshold", "off")
        assert tune_gc() == (12345, 7, 9) and gc.get_threshold() == (12345, 7, 9)  # "off" leaves them
    finally:
        gc.set_threshold(*before)


def test_now_us_matches_datetime_clock_and_pins():
    a = _clock.now_us()
    b = _clock.to_us(_clock.now())
    assert abs(b - a) < 2_000_000  # same CLOCK_REALTIME source
    pinned = _clock.from_us(1_767_225_600_123_456)
    _clock.set_clock(lambda: pinned)
    try:
        assert _clock.now_us() == 1_767_225_600_123_456
    finally:
        _clock.set_clock(None)


@pytest.mark.gpu
def test_store_worker_telemetry_counts_commands(cuda_device):
    from agent_hypervisor_amd.models.store import GovernanceStore

    st = GovernanceStore("cuda")
    try:
        i0 = st.info()
        for _ in range(50):
            st.flush()
        i1 = st.info()
        assert i1["worker_commands"] - i0["worker_commands"] >= 50
        assert i1["worker_busy_us"] > i0["worker_busy_us"]
    finally:
        st.close()
