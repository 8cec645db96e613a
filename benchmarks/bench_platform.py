#!/usr/bin/env python3
"""Platform floors on MI355X (SURVEY §7.2 Phase 0): the latencies every design
decision in this framework is priced against.

* ``launch``       — one tiny native kernel (``pipeline_advance``, 1 thread):
                     launch + stream sync round trip, and back-to-back issue rate;
* ``graph``        — the same kernel ×K captured in one hipGraph: replay + sync;
* ``event``        — hipEventRecord + hipEventSynchronize on an idle stream;
* ``d2h32``        — 32-byte device→pinned-host copy + sync (a Merkle root);
* ``pipeline1``    — one single-session batched pipeline launch + sync (what a
                     "GPU scalar path" would cost, vs the host scalar p50);
* ``allreduce``    — RCCL all-reduce latency by message size (8 B … 64 MB), only
                     when launched with ≥ 2 ranks by ``torch.distributed.run``.

Prints one JSON line per measurement (p50 over ``--iters`` samples, µs).
"""

from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import time

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def p50_us(fn, iters: int, warm: int = 20) -> float:
    for _ in range(warm):
        fn()
    ts = []
    for _ in range(iters):
        t0 = time.perf_counter_ns()
        fn()
        ts.append(time.perf_counter_ns() - t0)
    return statistics.median(ts) / 1e3


def emit(rank: int, **kw) -> None:
    if rank == 0:
        print(json.dumps(kw), flush=True)


def main() -> None:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--iters", type=int, default=2000)
    ap.add_argument("--graph-kernels", type=int, default=32)
    args = ap.parse_args()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)

    from agent_hypervisor_amd._native import C

    stream = torch.cuda.current_stream(dev)
    cursor = torch.zeros(3, dtype=torch.int64, device=dev)

    def tiny():
        C.pipeline_advance(cursor.data_ptr(), 1, 1 << 20, stream.cuda_stream)

    def launch_sync():
        tiny()
        stream.synchronize()

    emit(rank, what="launch+sync", p50_us=round(p50_us(launch_sync, args.iters), 2))
    n = 1000
    torch.cuda.synchronize()
    t0 = time.perf_counter_ns()
    for _ in range(n):
        tiny()
    torch.cuda.synchronize()
    emit(rank, what="launch back-to-back", us_per_launch=round((time.perf_counter_ns() - t0) / n / 1e3, 3))

    K = args.graph_kernels
    g = torch.cuda.CUDAGraph()
    side = torch.cuda.Stream(dev)
    side.wait_stream(stream)
    with torch.cuda.stream(side):
        with torch.cuda.graph(g, stream=side):
            for _ in range(K):
                C.pipeline_advance(cursor.data_ptr(), 1, 1 << 20, side.cuda_stream)
    stream.wait_stream(side)

    def graph_sync():
        g.replay()
        torch.cuda.current_stream(dev).synchronize()

    emit(rank, what=f"hipGraph replay ({K} kernels)+sync", p50_us=round(p50_us(graph_sync, args.iters), 2))

    ev = torch.cuda.Event()

    def event_sync():
        ev.record(stream)
        ev.synchronize()

    emit(rank, what="event record+sync", p50_us=round(p50_us(event_sync, args.iters), 2))

    src = torch.arange(8, dtype=torch.int32, device=dev)
    dst = torch.empty(8, dtype=torch.int32, pin_memory=True)

    def d2h():
        dst.copy_(src, non_blocking=True)
        stream.synchronize()

    emit(rank, what="D2H 32 B (pinned)+sync", p50_us=round(p50_us(d2h, args.iters), 2))

    from agent_hypervisor_amd.models.engine import GovernanceEngine

    eng = GovernanceEngine(device=str(dev), session_capacity=1 << 16, agent_capacity=1024, seed=3)
    eng.register_synthetic_agents(1000, seed=1)
    one = torch.zeros(1, dtype=torch.int32, device=dev)

    def pipe1():
        eng.run_pipeline(1, agents=one)
        stream.synchronize()

    p50 = round(p50_us(pipe1, max(200, args.iters // 4)), 2)
    emit(rank, what="batched pipeline, 1 session, launch+sync", p50_us=p50)

    if world > 1:
        for nbytes in (8, 1 << 10, 1 << 16, 1 << 20, 8 << 20, 64 << 20):
            t = torch.zeros(max(1, nbytes // 8), dtype=torch.float64, device=dev)

            def ar():
                dist.all_reduce(t)
                stream.synchronize()

            lat = p50_us(ar, 50 if nbytes >= (8 << 20) else 300, warm=10)
            emit(rank, what="RCCL all_reduce", world=world, bytes=nbytes, p50_us=round(lat, 2),
                 bus_GBps=round(2 * (world - 1) / world * nbytes / lat / 1e3, 2))
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
