"""N06 RCCL communicator on a real MI355X (world size 1 on the test box; the
multi-rank paths run in the driver's 8-GPU bench and the gloo harness)."""

from __future__ import annotations

import pytest
import torch

pytestmark = pytest.mark.gpu


def test_rccl_world1_collectives(cuda_device):
    from agent_hypervisor_amd.parallel.rccl import Communicator

    assert Communicator.version() > 0
    comm = Communicator.from_process_group(device=cuda_device.index or 0)
    assert comm.world == 1 and comm.rank == 0
    assert comm.async_error() == ""  # healthy (watchdog input, §5.3)
    x = torch.arange(10, dtype=torch.float64, device=cuda_device)
    assert torch.equal(comm.all_reduce(x.clone()), x)
    assert torch.equal(comm.all_reduce(x.clone(), op="max"), x)
    g = comm.all_gather(torch.arange(4, dtype=torch.int64, device=cuda_device))
    assert g.shape == (1, 4) and g[0].tolist() == [0, 1, 2, 3]
    assert torch.equal(comm.reduce_scatter(x.clone()), x)
    assert torch.equal(comm.broadcast(x.clone()), x)
    assert torch.equal(comm.all_to_all(x.clone()), x)
    with pytest.raises(ValueError):
        comm.all_reduce(torch.zeros(3))
    comm.destroy()
    with pytest.raises(RuntimeError):
        comm.all_reduce(x)


def test_rccl_all_reduce_inside_hip_graph(cuda_device):
    from agent_hypervisor_amd.parallel.rccl import Communicator

    comm = Communicator.from_process_group(device=cuda_device.index or 0)
    stats = torch.zeros(6, dtype=torch.int64, device=cuda_device)
    s = torch.cuda.Stream(cuda_device)
    s.wait_stream(torch.cuda.current_stream(cuda_device))
    with torch.cuda.stream(s):
        stats.add_(1)
        comm.all_reduce(stats, stream=s)
    torch.cuda.current_stream(cuda_device).wait_stream(s)
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        stats.add_(1)
        comm.all_reduce(stats)
    for _ in range(5):
        graph.replay()
    torch.cuda.synchronize(cuda_device)
    assert stats.tolist() == [6] * 6
    comm.destroy()


def test_abort_from_another_thread_during_collectives(cuda_device):
    """the watchdog aborts from its own thread while the issuing thread
    enqueues collectives; every call either completes or fails cleanly."""
    import threading
    import time

    from agent_hypervisor_amd.parallel.rccl import Communicator

    comm = Communicator.from_process_group(device=cuda_device.index or 0)
    x = torch.ones(1 << 16, dtype=torch.float64, device=cuda_device)
    outcomes = {"ok": 0, "aborted": 0}
    stop = threading.Event()

    def issuer():
        while not stop.is_set():
            try:
                comm.all_reduce(x)
                outcomes["ok"] += 1
            except RuntimeError as e:
                assert "aborted" in str(e) or "destroyed" in str(e)
                outcomes["aborted"] += 1
                break

    t = threading.Thread(target=issuer)
    t.start()
    time.sleep(0.05)
    comm.abort()  # from this (the watchdog's) thread
    stop.set()
    t.join(timeout=30)
    assert not t.is_alive()
    torch.cuda.synchronize(cuda_device)
    assert outcomes["ok"] > 0 and comm.async_error() in ("aborted", "destroyed")
    with pytest.raises(RuntimeError):
        comm.all_reduce(x)
