"""K03/K04 liability-stage variants on one GPU (config3 shapes):

* ``tiles``  — build_tiles (CSR → dense [S,16,16] fp64 tile in HBM) + bond_tiles
  (tile → MFMA column/row sums): round 1's MFMA path;
* ``csr``    — sigma_eff_csr (one lane per (session, vouchee), creation order,
  LDS-staged edges; σ_eff only);
* ``fused``  — bond_fused (CSR edges straight into v_mfma_f64_16x16x4_f64 as
  one-hot products: σ_eff + exposure + agent scatter, no tile).

``*_ns`` variants skip the agent-indexed exposure scatter (fp64 atomics into the
[A] vector), the like-for-like comparison with ``csr``;
* ``stream`` — sigma_eff_stream (K03 exact, register/DPP streaming form — the
  default ``sigma_eff_exact`` kernel since round 3);
* ``fused_gather`` — bond_fused + the AgentIndex segmented reduction (X01 input
  with no atomics, deterministic) instead of the in-kernel atomic scatter;
* ``exposure`` — ResidentBonds.exposure, the headline's K04 agent form
  (``--agents`` agents × ``--bond-degree`` edges, segmented LDS reduction);
* ``slash_split`` / ``slash_group`` — config5's storm (``--slash-sessions``
  sessions × 16 edges, 10 % slashed, σ_eff fused) in the round-3 split form and
  the round-2 single group pass.

Prints one JSON line per (variant, S) with µs per call (CUDA events, median of
``--iters``).  rocprofv3 --pmc FETCH_SIZE/WRITE_SIZE runs of this script give
the HBM traffic per kernel (profiles/liability_fused_r2.md)."""

from __future__ import annotations

import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from agent_hypervisor_amd.ops import liability as LI  # noqa: E402
from benchmarks.bench_configs import random_vouch_batch  # noqa: E402


def time_us(fn, iters: int) -> float:
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    out = []
    for _ in range(iters):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        b.synchronize()
        out.append(a.elapsed_time(b) * 1e3)
    return statistics.median(out)


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--sessions", type=int, nargs="*", default=[100_000, 1_250_000])
    ap.add_argument("--edges-per-session", type=int, default=8)
    ap.add_argument("--agents", type=int, default=1_000_000)
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--only", default="", help="comma list of variants (profiling)")
    ap.add_argument("--bond-degree", type=int, default=4)
    ap.add_argument("--slash-sessions", type=int, default=625_000)
    a = ap.parse_args()
    dev = torch.device("cuda")
    only = set(a.only.split(",")) if a.only else {"tiles", "tiles_ns", "csr", "stream", "fused", "fused_ns",
                                                  "fused_gather", "exposure", "slash_split", "slash_group"}
    if "exposure" in only:
        from agent_hypervisor_amd.ops.global_liability import ResidentBonds

        rb = ResidentBonds(a.agents, a.bond_degree, dev, seed=4242)
        out = torch.empty(a.agents, dtype=torch.float64, device=dev)
        us = time_us(lambda: rb.exposure(out), a.iters)
        print(json.dumps(dict(variant="exposure", agents=a.agents, edges=rb.edges, us=round(us, 2),
                              edges_per_us=round(rb.edges / us, 1),
                              hbm_gbps=round((rb.edges * 17 + a.agents * 16) / us / 1e3, 1))), flush=True)
        del rb
    for mode in ("split", "group"):
        if "slash_" + mode not in only:
            continue
        S5 = a.slash_sessions
        vb0 = random_vouch_batch(S5, 16, dev, seed=5)
        g5 = torch.Generator().manual_seed(9)
        tgt = torch.full((S5,), 255, dtype=torch.uint8)
        hit = torch.randperm(S5, generator=g5)[: S5 // 10]
        tgt[hit] = torch.randint(0, 16, (hit.numel(),), generator=g5, dtype=torch.uint8)
        tgt = tgt.to(dev)
        om5 = torch.full((S5,), 0.95, dtype=torch.float64, device=dev)
        sc0 = torch.rand((S5, 16), generator=g5, dtype=torch.float64).to(dev)
        n_it = a.iters + 3
        fresh = [(vb0.active.clone(), vb0.released_us.clone(), sc0.clone()) for _ in range(n_it)]

        def storm():
            act, rel, sc = fresh.pop()
            vb5 = LI.VouchBatch(vb0.offsets, vb0.voucher, vb0.vouchee, vb0.bonded, act, vb0.expiry_us, rel)
            return LI.slash(vb5, tgt, om5, sc, 1, clip_cap=16, zero_records=False, with_sigma_eff=True, mode=mode)

        us = time_us(storm, a.iters)
        print(json.dumps(dict(variant="slash_" + mode, sessions=S5, edges=S5 * 16, slashed=S5 // 10,
                              us=round(us, 2), edges_per_us=round(S5 * 16 / us, 1))), flush=True)
        del fresh, vb0
    for S in a.sessions:
        vb = random_vouch_batch(S, a.edges_per_session, dev, seed=1)
        g = torch.Generator(device=dev).manual_seed(2)
        sigma = torch.rand((S, 16), dtype=torch.float64, device=dev, generator=g)
        omega = torch.full((S,), 0.5, dtype=torch.float64, device=dev)
        members = torch.randint(0, a.agents, (S, 16), device=dev, generator=g)
        ax = torch.zeros(a.agents, dtype=torch.float64, device=dev)
        ref = LI.sigma_eff_exact(vb, sigma, omega, 0)
        E = S * a.edges_per_session
        res = {}
        if "tiles" in only:
            def tiles():
                t = LI.build_tiles(vb, 0)
                return LI.bond_tiles(t, sigma, omega, members=members, agent_exposure=ax)
            res["tiles"] = (time_us(tiles, a.iters), (tiles()[0] - ref).abs().max().item())
        if "tiles_ns" in only:
            def tiles_ns():
                return LI.bond_tiles(LI.build_tiles(vb, 0), sigma, omega)
            res["tiles_ns"] = (time_us(tiles_ns, a.iters), (tiles_ns()[0] - ref).abs().max().item())
        if "fused_ns" in only:
            def fused_ns():
                return LI.bond_fused(vb, sigma, omega, 0)
            res["fused_ns"] = (time_us(fused_ns, a.iters), (fused_ns()[0] - ref).abs().max().item())
        if "csr" in only:
            res["csr"] = (time_us(lambda: LI.sigma_eff_exact(vb, sigma, omega, 0, kernel="csr"), a.iters), 0.0)
        if "stream" in only:
            res["stream"] = (time_us(lambda: LI.sigma_eff_exact(vb, sigma, omega, 0, kernel="stream"), a.iters),
                             (LI.sigma_eff_exact(vb, sigma, omega, 0, kernel="stream") - ref).abs().max().item())
        if "fused_gather" in only:
            aidx = LI.agent_index(vb, members, a.agents)

            def fused_gather():
                return LI.bond_fused(vb, sigma, omega, 0, agent_exposure=ax, agent_idx=aidx)
            res["fused_gather"] = (time_us(fused_gather, a.iters), (fused_gather()[0] - ref).abs().max().item())
        if "fused" in only:
            def fused():
                return LI.bond_fused(vb, sigma, omega, 0, members=members, agent_exposure=ax)
            res["fused"] = (time_us(fused, a.iters), (fused()[0] - ref).abs().max().item())
        if "admit" in only or not a.only:  # K05: 4 vouch requests per session against the resident edges
            g2 = torch.Generator(device=dev).manual_seed(3)
            R = 4 * S
            r_off = (torch.arange(S + 1, device=dev) * 4).to(torch.int32)
            rv = torch.randint(0, 16, (R,), device=dev, generator=g2).to(torch.uint8)
            re_ = torch.randint(0, 16, (R,), device=dev, generator=g2).to(torch.uint8)
            rs = torch.rand(R, dtype=torch.float64, device=dev, generator=g2) * 0.7 + 0.3
            rp = torch.full((R,), 0.1, dtype=torch.float64, device=dev)
            us = time_us(lambda: LI.vouch_admit(vb, r_off, rv, re_, rs, rp, 0), a.iters)
            print(json.dumps(dict(variant="vouch_admit", sessions=S, edges=E, requests=R, us=round(us, 2),
                                  requests_per_us=round(R / us, 1))), flush=True)
        for k, (us, err) in res.items():
            print(json.dumps(dict(variant=k, sessions=S, edges=E, us=round(us, 2),
                                  edges_per_us=round(E / us, 1), max_abs_err_vs_csr=err,
                                  outputs={"csr": "sigma_eff", "stream": "sigma_eff"}.get(k, "sigma_eff+exposure" + (
                                      "" if k.endswith("_ns") else "+agent_vector")))),
                  flush=True)


if __name__ == "__main__":
    main()
