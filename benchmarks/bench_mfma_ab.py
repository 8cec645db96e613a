#!/usr/bin/env python3
"""σ_eff / exposure at the config3 shape: fp64 MFMA path vs the exact VALU kernels.

config3: 100k sessions × 16 participant rows, 8 vouch edges per
session, 1M-agent exposure vector.  Both paths produce σ_eff [S,16] and the
agent-indexed exposure [A]:

* ``mfma``  — ``bond_fused`` (CSR edges → ``v_mfma_f64_16x16x4_f64`` with a
  one-hot operand: the per-session row/column sums) + the segmented agent gather;
* ``exact`` — ``sigma_eff_exact`` (creation-order sums, bit-identical to the
  reference) + per-session exposure rows (one VALU scatter-add over the live
  edges) and the same agent gather.

Prints one JSON line per path (median µs over ``--iters`` CUDA-event timings)
and the max |Δσ_eff| in ulps between them.
"""

from __future__ import annotations

import argparse
import json
import os
import statistics
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--sessions", type=int, default=100_000)
    ap.add_argument("--edges", type=int, default=8)
    ap.add_argument("--agents", type=int, default=1_000_000)
    ap.add_argument("--iters", type=int, default=200)
    ap.add_argument("--device", default="cuda")
    args = ap.parse_args()
    from agent_hypervisor_amd.ops import liability as LI
    from benchmarks.bench_configs import random_vouch_batch

    dev = torch.device(args.device)
    S, A = args.sessions, args.agents
    vb = random_vouch_batch(S, args.edges, dev, seed=3)
    g = torch.Generator(device=dev).manual_seed(5)
    members = torch.randint(0, A, (S, 16), device=dev, generator=g)
    sigma = torch.rand((S, 16), dtype=torch.float64, device=dev, generator=g)
    omega = torch.full((S,), 0.5, dtype=torch.float64, device=dev)
    idx = LI.agent_index(vb, members, A)
    expo = torch.zeros(A, dtype=torch.float64, device=dev)

    def mfma():
        se, ex, _ = LI.bond_fused(vb, sigma, omega, 0, agent_exposure=expo, agent_idx=idx)
        return se

    counts = (vb.offsets[1:] - vb.offsets[:-1]).to(torch.int64)
    row = torch.repeat_interleave(torch.arange(S, device=dev, dtype=torch.int64), counts) * 16 + \
        vb.voucher.to(torch.int64)
    live = vb.active.bool() & (vb.expiry_us < 0)

    def exact():
        se = LI.sigma_eff_exact(vb, sigma, omega, 0)
        ex = torch.zeros(S * 16, dtype=torch.float64, device=dev)
        ex.index_add_(0, row, torch.where(live, vb.bonded, torch.zeros_like(vb.bonded)))  # K04 rows
        LI.agent_gather(idx, ex.view(S, 16), expo)
        return se

    def timed(fn):
        for _ in range(10):
            fn()
        if dev.type != "cuda":
            return None
        ts = []
        for _ in range(args.iters):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            fn()
            b.record()
            b.synchronize()
            ts.append(a.elapsed_time(b) * 1e3)
        return statistics.median(ts)

    t_m, t_e = timed(mfma), timed(exact)
    a, b = mfma(), exact()
    ulp = ((a.view(torch.int64) - b.view(torch.int64)).abs().max()).item()
    for name, t in (("mfma", t_m), ("exact", t_e)):
        print(json.dumps({"bench": "sigma_exposure_config3", "path": name, "sessions": S, "edges": args.edges,
                          "agents": A, "median_us": t, "max_ulp_vs_other": ulp}))


if __name__ == "__main__":
    main()
