#!/usr/bin/env python3
"""Headline benchmark: the reference's ``full_governance_pipeline`` on MI355X.

BASELINE.json metric: "p50 pipeline latency (µs) + session-ops/sec,
bench_hypervisor.py at 1/2/4/8 GPU".  One *session-op* is one complete run of the
reference pipeline (bench_hypervisor.py:217-239) for one session: create → join
(σ ring gate) → activate → 3 audit deltas (canonical JSON + SHA-256 Merkle chain)
→ saga create/add/execute step → terminate (Merkle root, commitment, bond
release, GC, archive).

Each timed step runs that pipeline for ``--sessions`` new sessions per GPU in one
gfx950 launch (device-resident tables, device-minted ids, synthetic agents with
random-init σ), then a cross-rank RCCL all-reduce of the step's governance
counters (collective X04) — weak scaling, sessions sharded data-parallel.

Also reported (not the headline value):
* ``device_p50_us`` — p50 of the single-session pipeline through the public
  ``Hypervisor(device="cuda")`` API, reference harness methodology (2,000
  iterations after warm-up): every state change, ring gate, audit digest,
  Merkle root, bond release and saga transition is executed by the resident
  gfx950 store worker (hypervisor/_device.py, csrc/hip/store_worker.hip);
* ``scalar_p50_us`` — the same harness on the pure host engines (CPU only);
* ``batch_p50_ms`` — p50 wall time of one synchronised pipeline step.

``vs_baseline`` divides the batched GPU throughput by the reference's
single-threaded Python pipeline rate — a capability ratio, not a like-for-like
one; ``device_vs_baseline_p50`` compares like with like (one session, public
API, same harness).

Launch: ``python bench.py`` (1 GPU) or via ``torch.distributed.run`` for N GPUs.
"""

from __future__ import annotations

import argparse
import asyncio
import json
import os
import statistics
import sys
import time

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

BASELINE_OPS = 2983.0  # published full_governance_pipeline throughput
BASELINE_P50_US = 267.5
METRIC = "p50 pipeline latency (µs) + session-ops/sec, bench_hypervisor.py at 1/2/4/8 GPU"


def scalar_pipeline_p50(iters: int = 2000, device: str = "host") -> tuple[float, float]:
    """Reference-harness timing of the public-API pipeline (bench_hypervisor.py:217-239).

    ``device="host"``: pure host engines; ``device="cuda"``: the device-authoritative
    store (every call is a command to the gfx950 worker)."""
    from hypervisor import Hypervisor, SessionConfig
    from hypervisor.audit.delta import VFSChange

    async def one():
        hv = Hypervisor(device=device)
        s = await hv.create_session(config=SessionConfig(enable_audit=True), creator_did="did:mesh:admin")
        sid = s.sso.session_id
        await hv.join_session(sid, "did:mesh:a", sigma_raw=0.8)
        await hv.activate_session(sid)
        for i in range(3):
            s.delta_engine.capture("did:mesh:a", [VFSChange(path=f"/f{i}", operation="add", content_hash=f"h{i}")])
        saga = s.saga.create_saga(sid)
        step = s.saga.add_step(saga.saga_id, "action", "did:mesh:a", "/api/action")
        await s.saga.execute_step(saga.saga_id, step.step_id, executor=lambda: asyncio.sleep(0))
        await hv.terminate_session(sid)

    async def run():
        times = []
        for _ in range(min(100, iters // 10)):
            await one()
        for _ in range(iters):
            t0 = time.perf_counter_ns()
            await one()
            times.append(time.perf_counter_ns() - t0)
        return times

    times = asyncio.run(run())
    return statistics.median(times) / 1000.0, statistics.mean(times) / 1000.0


def main() -> None:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--sessions", type=int, default=1 << 20, help="sessions per GPU per step")
    ap.add_argument("--agents", type=int, default=1 << 20, help="synthetic agents per GPU")
    ap.add_argument("--deltas", type=int, default=3)
    ap.add_argument("--scalar-iters", type=int, default=2000)
    ap.add_argument("--no-scalar", action="store_true")
    ap.add_argument("--graph", action="store_true",
                    help="replay each step from a captured hipGraph (device cursor + RCCL counters)")
    ap.add_argument("--device", choices=("cuda", "cpu"), default="cuda",
                    help="cpu runs the host twin of the kernel over gloo (multi-process CPU rehearsal)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # AHV_BENCH_FORCE_DIST=1 (under torch.distributed.run) takes the multi-rank path
    # — process group, async RCCL counter all-reduce, barriers, max-over-ranks —
    # even with one rank, so the code the 8-GPU run executes is exercised on 1 GPU.
    multi = world > 1 or os.environ.get("AHV_BENCH_FORCE_DIST") == "1"
    if multi:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    if args.device == "cuda":
        torch.cuda.set_device(local)
        dev = torch.device("cuda", local)
    else:
        dev = torch.device("cpu")
    if multi:
        if dev.type == "cuda":
            dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)
        else:
            dist.init_process_group("gloo", rank=rank, world_size=world)

    def sync():
        if dev.type == "cuda":
            torch.cuda.synchronize(dev)

    from agent_hypervisor_amd.models.engine import GovernanceEngine
    from agent_hypervisor_amd.parallel.collectives import allreduce_stats  # noqa: F401 (graph mode)

    S = args.sessions
    eng = GovernanceEngine(
        device=str(dev), session_capacity=2 * S, agent_capacity=args.agents, seed=0x5EED0000 + rank
    )
    eng.register_synthetic_agents(args.agents, seed=1000 + rank, prefix=f"did:mesh:r{rank}-agent-")
    g = torch.Generator(device=dev).manual_seed(77 + rank)
    stats = torch.zeros(6, dtype=torch.int64, device=dev)

    # X04 counters: double-buffered so step i's all-reduce (RCCL, on its own
    # stream) overlaps step i+1's pipeline kernel; a buffer is reused only after
    # its collective from two steps back has completed (a stream wait, no host sync).
    bufs = [torch.zeros(6, dtype=torch.int64, device=dev) for _ in range(2)]
    works: list = [None, None]
    it = [0]

    def step():
        b = it[0] & 1
        it[0] += 1
        if works[b] is not None:
            works[b].wait()
        st = bufs[b]
        st.zero_()
        agents = torch.randint(0, args.agents, (S,), device=dev, dtype=torch.int32, generator=g)
        eng.run_pipeline(S, agents=agents, deltas=args.deltas, stats=st)
        works[b] = dist.all_reduce(st, op=dist.ReduceOp.SUM, async_op=True) if multi else None
        return st

    def drain():
        for k in range(2):
            if works[k] is not None:
                works[k].wait()
                works[k] = None

    if args.graph:
        from agent_hypervisor_amd.runtime.graphs import PipelineGraph

        reduce = None
        if multi and dev.type == "cuda":
            from agent_hypervisor_amd.parallel.rccl import Communicator

            comm = Communicator.from_process_group(device=local)
            reduce = comm.all_reduce
        elif multi:
            reduce = allreduce_stats
        buf = torch.zeros(S, dtype=torch.int32, device=dev)
        pg = PipelineGraph(eng, S, buf, deltas=args.deltas, stats=stats,
                           refresh_agents=lambda: buf.random_(0, args.agents), reduce=reduce)

        def step():  # noqa: F811 - graph-replay form of the same step
            pg.step()
            return stats

        def drain():  # noqa: F811 - the graph's collective is in-stream
            pass

    for _ in range(args.warmup):
        step()
    drain()
    sync()

    # per-step latency distribution (synchronised steps, untimed for throughput)
    lat = []
    for _ in range(max(3, min(10, args.steps))):
        t0 = time.perf_counter()
        step()
        drain()
        sync()
        lat.append(time.perf_counter() - t0)

    if multi:
        dist.barrier()
    sync()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        last = step()
    drain()
    sync()
    if multi:
        dist.barrier()
    elapsed = time.perf_counter() - t0

    if multi:
        e = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(e, op=dist.ReduceOp.MAX)
        elapsed = float(e.item())
    totals = last.cpu().tolist()

    scalar_p50 = scalar_mean = device_p50 = device_mean = None
    if rank == 0 and not args.no_scalar:
        scalar_p50, scalar_mean = scalar_pipeline_p50(args.scalar_iters, "host")
        if dev.type == "cuda":
            device_p50, device_mean = scalar_pipeline_p50(args.scalar_iters, "cuda")

    if rank == 0:
        total_sessions = S * world * args.steps
        value = total_sessions / elapsed
        out = {
            "metric": METRIC,
            "value": round(value, 1),
            "unit": "session-ops/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1000.0, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": round(value / BASELINE_OPS, 2),
            "dtype": "fp64",
            "data": "synthetic",
            "config": {
                "model": "full_governance_pipeline",
                "global_batch": S * world,
                "seq_len": args.deltas,
                "parallelism": f"dp{world}",
                "sessions_per_gpu": S,
                "agents_per_gpu": args.agents,
                "deltas_per_session": args.deltas,
            },
            "batch_p50_ms": round(statistics.median(lat) * 1000.0, 4),
            "vs_baseline_note": "batched GPU throughput / single-threaded Python reference rate (not like-for-like)",
            "device_p50_us": round(device_p50, 2) if device_p50 is not None else None,
            "device_mean_us": round(device_mean, 2) if device_mean is not None else None,
            "device_vs_baseline_p50": round(BASELINE_P50_US / device_p50, 3) if device_p50 else None,
            "scalar_p50_us": round(scalar_p50, 2) if scalar_p50 is not None else None,
            "scalar_mean_us": round(scalar_mean, 2) if scalar_mean is not None else None,
            "scalar_vs_baseline_p50": round(BASELINE_P50_US / scalar_p50, 2) if scalar_p50 else None,
            "last_step_counters": dict(zip(["sessions", "ok", "participants", "deltas", "commits", "archived"], totals)),
        }
        print(json.dumps(out), flush=True)
    if multi:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
