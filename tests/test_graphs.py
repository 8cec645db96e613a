"""N07/N09: cursor-driven pipeline batches and the hipGraph step runner.

CPU: the eager host-twin sequence (clock → pipeline → advance) must write the
same rows as ordinary ``run_pipeline`` calls.  GPU: graph replays must equal
the host twin for the replayed cursor (same ids, timestamps and digests)."""

from __future__ import annotations

from datetime import datetime, timezone

import pytest
import torch

from agent_hypervisor_amd.models.engine import GovernanceEngine
from agent_hypervisor_amd.runtime.graphs import PipelineGraph
from hypervisor import _clock

T0 = datetime(2026, 6, 1, 9, 0, tzinfo=timezone.utc)


def _engine(device, seed=11, capacity=1000):
    eng = GovernanceEngine(device=device, session_capacity=capacity, agent_capacity=256, seed=seed)
    eng.register_synthetic_agents(200, seed=3)
    return eng


def test_cursor_path_matches_eager_cpu():
    _clock.set_clock(lambda: T0)
    n = 96
    a = _engine("cpu")
    agents = (torch.arange(n, dtype=torch.int32) * 7) % 200
    pg = PipelineGraph(a, n, agents.clone(), stats=torch.zeros(6, dtype=torch.int64))
    assert not pg.use_graph
    for _ in range(3):
        pg.step()
    assert pg.stats.tolist()[:2] == [n, n]
    last = pg.last_batch()
    b = _engine("cpu")
    for _ in range(3):
        ref = b.run_pipeline(n, agents=agents, deltas=3)
    assert last.slot_base == ref.slot_base and last.now_us == ref.now_us == _clock.to_us(T0)
    assert torch.equal(last.roots(), ref.roots())
    assert last.session_id(5) == ref.session_id(5)
    assert last.materialize(0).delta_engine.verify_chain()
    # eager calls after graph steps continue from the mirrored counters
    nxt = a.run_pipeline(8, agents=agents[:8])
    assert nxt.slot_base == (3 * n) % 1000


def test_wraparound_cursor_cpu():
    _clock.set_clock(lambda: T0)
    eng = GovernanceEngine(device="cpu", session_capacity=100, agent_capacity=64, seed=1)
    eng.register_synthetic_agents(50)
    pg = PipelineGraph(eng, 64, torch.zeros(64, dtype=torch.int32))
    pg.step()
    pg.step()
    assert pg.cursor[0].item() == 28 and pg.last_batch().slot_base == 64


@pytest.mark.gpu
def test_graph_replay_matches_host_twin(cuda_device):
    n = 4096
    dev_eng = _engine(str(cuda_device), seed=99, capacity=10_000)
    agents = torch.randint(0, 200, (n,), dtype=torch.int32, device=cuda_device)
    stats = torch.zeros(6, dtype=torch.int64, device=cuda_device)
    pg = PipelineGraph(dev_eng, n, agents, stats=stats)
    assert pg.use_graph and pg.graph is not None
    for _ in range(3):
        pg.step()
    torch.cuda.synchronize(cuda_device)
    assert stats.tolist()[:2] == [n, n]
    last = pg.last_batch()
    host = _engine("cpu", seed=99, capacity=10_000)
    host._next_slot, host._id_counter = last.slot_base, last.id_base
    ref = host.run_pipeline(n, agents=agents.cpu(), deltas=3, now_us=last.now_us)
    assert torch.equal(last.roots().cpu(), ref.roots())
    assert last.session_id(17) == ref.session_id(17)
    # device "now" is close to host UTC (calibrated wall clock)
    assert abs(last.now_us - _clock.now_us()) < 5_000_000
