#!/usr/bin/env python3
"""Capacity sweep: HBM-resident liability graphs and pipeline batches far beyond the
headline's sizes (SURVEY §7.1 item 5 sizing: tens of millions of agent records
resident per GPU, 288 GB of HBM3E).

For each agent count A (degree-4 resident vouch graph, 4·A edges) it reports the
resident bytes and the time of K04 agent exposure (atomic-free segmented sum over
every edge) and of a K06 slash-clip stage over 1 % of the agents; for each session
batch S the time of one full governance-pipeline launch (the headline kernel).

    python benchmarks/bench_capacity.py --agents 1e6 16e6 64e6 --sessions 1e6 4e6 8e6
"""

from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _timed(fn, reps: int) -> float:
    """Median wall time of ``fn`` (synchronised) over ``reps`` runs, in µs."""
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    return statistics.median(ts) * 1e6


def liability(A: int, reps: int) -> dict:
    from agent_hypervisor_amd.ops.global_liability import ResidentBonds

    dev = torch.device("cuda")
    bonds = ResidentBonds(A, 4, dev, seed=1)
    out = torch.zeros(A, dtype=torch.float64, device=dev)
    k = max(1, A // 100)
    ids = torch.randint(0, A, (k,), dtype=torch.int32, device=dev, generator=torch.Generator(device=dev).manual_seed(2))
    cap = 16 * k
    pid = torch.full((cap,), -1, dtype=torch.int32, device=dev)
    pf = torch.ones(cap, dtype=torch.float64, device=dev)
    cur = torch.zeros(1, dtype=torch.int64, device=dev)
    t_expo = _timed(lambda: bonds.exposure(out), reps)
    touched = A * 4 * (8 + 1 + 8) + (A + 1) * 8 + A * 8  # bonded, active, expiry, offsets, out

    def clip():
        bonds.active.fill_(1)
        cur.zero_()
        bonds.slash_clip(ids, 0.95, pid, pf, cur)

    t_fill = _timed(lambda: bonds.active.fill_(1), reps)
    t_clip = max(0.0, _timed(clip, reps) - t_fill)
    r = {"agents": A, "edges": bonds.edges, "resident_bytes": bonds.nbytes, "exposure_us": round(t_expo, 1),
         "exposure_TBps": round(touched / (t_expo * 1e-6) / 1e12, 2), "slash_k": k, "slash_clip_us": round(t_clip, 1),
         "clip_pairs": int(cur.item())}
    del bonds, out
    torch.cuda.empty_cache()
    return r


def pipeline(S: int, reps: int) -> dict:
    from agent_hypervisor_amd.models.engine import GovernanceEngine

    dev = torch.device("cuda")
    A = 1 << 20
    eng = GovernanceEngine(device=str(dev), session_capacity=2 * S, agent_capacity=A, seed=3)
    eng.register_synthetic_agents(A, seed=4)
    stats = torch.zeros(6, dtype=torch.int64, device=dev)
    g = torch.Generator(device=dev).manual_seed(5)
    agents = torch.randint(0, A, (S,), dtype=torch.int32, device=dev, generator=g)

    def step():
        stats.zero_()
        eng.run_pipeline(S, agents=agents, deltas=3, stats=stats)

    t = _timed(step, reps)
    ok = int(stats[1].item())
    r = {"sessions": S, "ms_per_launch": round(t / 1e3, 3), "sessions_per_s": round(S / (t * 1e-6), 1), "ok": ok == S}
    del eng
    torch.cuda.empty_cache()
    return r


def main() -> None:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--agents", type=float, nargs="*", default=[1e6, 16e6, 64e6])
    ap.add_argument("--sessions", type=float, nargs="*", default=[1 << 20, 1 << 22, 1 << 23])
    ap.add_argument("--reps", type=int, default=10)
    args = ap.parse_args()
    if not torch.cuda.is_available():
        raise SystemExit("bench_capacity needs a HIP device")
    for A in args.agents:
        print(json.dumps({"what": "liability", **liability(int(A), args.reps)}), flush=True)
    for S in args.sessions:
        print(json.dumps({"what": "pipeline", **pipeline(int(S), args.reps)}), flush=True)
    free, total = torch.cuda.mem_get_info()
    print(json.dumps({"what": "device", "hbm_total_gb": round(total / 2**30, 1),
                      "max_allocated_gb": round(torch.cuda.max_memory_allocated() / 2**30, 2)}), flush=True)


if __name__ == "__main__":
    main()
