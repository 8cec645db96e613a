"""N08 device event ring: the pipeline kernel (and its host twin) append the
same lifecycle events the scalar facade publishes; drain into the event bus."""

from __future__ import annotations

import pytest
import torch

from agent_hypervisor_amd.models.engine import GovernanceEngine
from agent_hypervisor_amd.runtime.events import DeviceEventRing
from hypervisor.observability.event_bus import EVENT_CODE, EventType, HypervisorEventBus

SCALAR_SEQUENCE = ["session.created", "session.joined", "ring.assigned", "session.activated",
                   "session.terminated", "audit.committed", "audit.gc_collected", "session.archived"]


def test_event_codes_match_python_enum():
    import re

    import os

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    text = open(os.path.join(root, "csrc", "include", "ahv", "events.h")).read()
    for name, code in re.findall(r"EV_([A-Z_]+) = (\d+)", text):
        assert EVENT_CODE[EventType[name]] == int(code), name


def _run(device, n=300, cap=40_000):
    eng = GovernanceEngine(device=device, session_capacity=1024, agent_capacity=512, seed=5)
    eng.register_synthetic_agents(400, seed=2)
    ring = DeviceEventRing(cap, device)
    b = eng.run_pipeline(n, deltas=3, events=ring, now_us=1_700_000_000_000_000)
    return eng, ring, b


def test_host_twin_emits_scalar_sequence():
    eng, ring, b = _run("cpu")
    assert ring.pending == 300 * 8 and ring.dropped == 0
    bus = HypervisorEventBus()
    evs = ring.drain(eng, bus)
    assert len(evs) == 2400 and bus.event_count == 2400 and ring.pending == 0
    sid = b.session_id(11)
    seq = [e.event_type.value for e in bus.query_by_session(sid)]
    assert seq == SCALAR_SEQUENCE
    joined = bus.query(session_id=sid, event_type=EventType.RING_ASSIGNED)[0]
    assert joined.agent_did.startswith("did:mesh:agent-") and joined.payload["ring"] in (2, 3)


def test_ring_overflow_counts_drops():
    eng, ring, _ = _run("cpu", n=100, cap=50)  # rounds up to 64 records = 64 segments of 1
    # sessions 0..63 append to segment 0, 64..99 to segment 1 (workgroup residues)
    assert ring.pending == 2 and ring.dropped == 798
    ring.drain(eng)
    assert ring.total_dropped == 798


@pytest.mark.gpu
def test_device_ring_matches_host(cuda_device):
    n = 50_000
    eng_d = GovernanceEngine(device=str(cuda_device), session_capacity=n, agent_capacity=4096, seed=9)
    eng_d.register_synthetic_agents(4096, seed=1)
    eng_h = GovernanceEngine(device="cpu", session_capacity=n, agent_capacity=4096, seed=9)
    eng_h.register_synthetic_agents(4096, seed=1)
    agents = torch.randint(0, 4096, (n,), dtype=torch.int32)
    rd, rh = DeviceEventRing(8 * n * 2, cuda_device), DeviceEventRing(8 * n * 2, "cpu")
    eng_d.run_pipeline(n, agents=agents.to(cuda_device), events=rd, now_us=123)
    eng_h.run_pipeline(n, agents=agents, events=rh, now_us=123)
    torch.cuda.synchronize(cuda_device)
    assert rd.pending == rh.pending == 8 * n
    sd, sh = rd.snapshot(), rh.snapshot()
    # device order differs (wave reservations); compare as sorted record sets
    key = lambda s: torch.stack([s["slot"].to(torch.int64), s["type"].to(torch.int64), s["ts_us"],
                                 s["agent"].to(torch.int64), s["aux"].to(torch.int64)], 1)
    a = key(sd)
    b = key(sh)
    a = a[torch.argsort(a[:, 0] * 64 + a[:, 1])]
    b = b[torch.argsort(b[:, 0] * 64 + b[:, 1])]
    assert torch.equal(a, b)
