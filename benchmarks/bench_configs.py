#!/usr/bin/env python3
"""Batched device benchmarks for BASELINE.json configs 2–5.

  config2  10k concurrent sessions: full governance pipeline (ring gate +
           Merkle audit) + σ_eff on fp64 MFMA bond tiles + ring re-gate,
           hipGraph-replayed — latency per batch and sessions/s
  config3  1M agents / 100k sessions sharded over the ranks (DP) with the
           cross-session vouch exposure all-reduce (X01, [A] fp64 over RCCL)
  config4  saga orchestrator: 10-step compensation chains, fused kernel and
           the hipGraph-captured step loop
  config5  liability slash storm: every session slashed (K06 cascade) and its
           remaining bonds released (K07) — all 10M resident bonds change
           state, device-counted — + σ_eff recompute + full delta re-chain (K08)
           and Merkle roots (K09) of every session; config5_subset: the 10 %
           storm with only the touched sessions re-chained

Each prints one JSON line per measurement.  ``--device cpu`` runs the host
twins at small scale (harness check).  Multi-rank: launch with
``torch.distributed.run`` (config3 is the one that communicates).
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

from agent_hypervisor_amd.models.engine import GovernanceEngine  # noqa: E402
from agent_hypervisor_amd.models.saga_engine import SagaBatchEngine, SagaOutcomes  # noqa: E402
from agent_hypervisor_amd.ops import audit as A  # noqa: E402
from agent_hypervisor_amd.ops import liability as LI  # noqa: E402
from agent_hypervisor_amd.ops import rings as R  # noqa: E402
from agent_hypervisor_amd.parallel import agent_shard as AS  # noqa: E402
from agent_hypervisor_amd.parallel import collectives as X  # noqa: E402
from agent_hypervisor_amd.parallel.directory import shard_counts  # noqa: E402
from agent_hypervisor_amd.runtime.graphs import PipelineGraph  # noqa: E402

f64, u8, i32, i64 = torch.float64, torch.uint8, torch.int32, torch.int64


class Ctx:
    def __init__(self, device: str):
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        local = int(os.environ.get("LOCAL_RANK", "0"))
        if device == "cuda":
            torch.cuda.set_device(local)
            self.dev = torch.device("cuda", local)
        else:
            self.dev = torch.device("cpu")
        if self.world > 1 and not dist.is_initialized():
            if self.dev.type == "cuda":
                dist.init_process_group("nccl", rank=self.rank, world_size=self.world, device_id=self.dev)
            else:
                dist.init_process_group("gloo", rank=self.rank, world_size=self.world)

    def sync(self):
        if self.dev.type == "cuda":
            torch.cuda.synchronize(self.dev)

    def barrier(self):
        if self.world > 1:
            dist.barrier()

    def timed(self, fn, steps: int, warmup: int) -> tuple[float, list[float]]:
        for _ in range(warmup):
            fn()
        self.sync()
        lat = []
        for _ in range(max(3, min(10, steps))):
            t0 = time.perf_counter()
            fn()
            self.sync()
            lat.append(time.perf_counter() - t0)
        self.barrier()
        self.sync()
        t0 = time.perf_counter()
        for _ in range(steps):
            fn()
        self.sync()
        self.barrier()
        el = time.perf_counter() - t0
        if self.world > 1:
            e = torch.tensor([el], dtype=f64, device=self.dev)
            dist.all_reduce(e, op=dist.ReduceOp.MAX)
            el = float(e.item())
        return el, lat

    def emit(self, **kw):
        if self.rank == 0:
            kw.setdefault("n_gpus", self.world)
            kw.setdefault("device", str(self.dev))
            print(json.dumps(kw), flush=True)


def random_vouch_batch(S: int, edges_per_session: int, dev, seed: int = 0) -> LI.VouchBatch:
    g = torch.Generator().manual_seed(seed)
    E = S * edges_per_session
    vr = torch.randint(0, 16, (E,), generator=g, dtype=torch.int64)
    ve = (vr + torch.randint(1, 16, (E,), generator=g)) % 16  # never self
    return LI.VouchBatch(
        offsets=(torch.arange(S + 1, dtype=i64) * edges_per_session).to(i32).to(dev),
        voucher=vr.to(u8).to(dev), vouchee=ve.to(u8).to(dev),
        bonded=(torch.rand(E, generator=g, dtype=f64) * 0.2).to(dev),
        active=torch.ones(E, dtype=u8, device=dev), expiry_us=torch.full((E,), -1, dtype=i64, device=dev),
        released_us=torch.zeros(E, dtype=i64, device=dev),
    )


# ------------------------------------------------------------------ config 2


def config2(ctx: Ctx, args):
    S = args.sessions or 10_000
    eng = GovernanceEngine(device=str(ctx.dev), session_capacity=4 * S, agent_capacity=max(S, 1024), seed=0xC2)
    eng.register_synthetic_agents(max(S, 1024), seed=2)
    agents = torch.randint(0, max(S, 1024), (S,), dtype=i32, device=ctx.dev)
    stats = torch.zeros(6, dtype=i64, device=ctx.dev)
    g = torch.Generator(device="cpu").manual_seed(3)
    tiles = (torch.rand((S, 16, 16), generator=g, dtype=f64) * 0.05).to(ctx.dev)
    sigma = torch.rand((S, 16), generator=g, dtype=f64).to(ctx.dev)
    omega = torch.full((S,), 0.5, dtype=f64, device=ctx.dev)

    def liability_tail():
        se, expo, _ = LI.bond_tiles(tiles, sigma, omega)
        R.ring_gate(se.reshape(-1))

    # (Running the σ_eff + ring-gate stage on a second stream beside the pipeline
    # measured slower — 0.154 vs 0.136 ms — the cross-stream event waits cost more
    # than the ~15 µs stage they would hide; one stream it is, captured with the
    # pipeline in one graph: pipeline kernel, epilogue, σ_eff tiles, ring gate.)
    pg = PipelineGraph(eng, S, agents, stats=stats, tail=liability_tail, fused=not args.unfused_graph)

    def step():
        pg.step()

    el, lat = ctx.timed(step, args.steps, args.warmup)
    ctx.emit(config="config2", what="pipeline+sigma_eff(MFMA)+ring_gate", sessions_per_step=S,
             batch_p50_ms=statistics.median(lat) * 1e3, ms_per_step=el / args.steps * 1e3,
             sessions_per_s=S * ctx.world * args.steps / el, graph=pg.use_graph,
             ok=int(stats[1].item()) == S)


# ------------------------------------------------------------------ config 3


def config3(ctx: Ctx, args):
    A_ = args.agents or 1_000_000
    S = shard_counts(args.sessions or 100_000, ctx.world)[ctx.rank]
    eng = GovernanceEngine(device=str(ctx.dev), session_capacity=4 * S, agent_capacity=A_, seed=0xC3 + ctx.rank)
    eng.register_synthetic_agents(A_, seed=7)  # the same global agent population on every rank
    gen = torch.Generator(device=ctx.dev).manual_seed(11 + ctx.rank)
    stats = torch.zeros(6, dtype=i64, device=ctx.dev)
    vb = random_vouch_batch(S, 8, ctx.dev, seed=ctx.rank)
    # participants of each session → global agent ids (for the agent-indexed exposure view)
    members = torch.randint(0, A_, (S, 16), device=ctx.dev, generator=gen)
    sigma = eng.agents.sigma[members]
    omega = torch.full((S,), 0.5, dtype=f64, device=ctx.dev)
    # double-buffered exposure view: step i's exchange runs on a side stream (P03)
    # while step i+1's pipeline kernel runs; owner mode reduce-scatters so each
    # rank keeps only the agents it owns (P02), half the all-reduce traffic
    exposure = [torch.zeros(A_, dtype=f64, device=ctx.dev) for _ in range(2)]
    comm = [AS.OverlappedCollective(ctx.dev) for _ in range(2)]
    owned = {}
    owner_reduce = not args.allreduce_exposure
    exchange = (lambda t: owned.__setitem__("view", AS.reduce_to_owners(t))) if owner_reduce \
        else X.allreduce_exposure
    it = [0]
    # P03: the liability stage (tile build + fp64 MFMA σ_eff/exposure) does not
    # read this step's pipeline output, and 100 k sessions fill only half the
    # GPU's wave slots, so the stage runs on a second stream beside the pipeline
    side = torch.cuda.Stream(ctx.dev) if ctx.dev.type == "cuda" else None

    def liability_stage(cur):
        comm[cur].wait()  # buffer reuse: the exchange from two steps ago is done
        exposure[cur].zero_()
        # σ_eff / exposure on fp64 MFMA; exposure scattered into the agent vector in-kernel
        if args.tiles:  # round-1 pair: dense tile through HBM, then MFMA sums
            LI.bond_tiles(LI.build_tiles(vb, 0), sigma, omega, members=members, agent_exposure=exposure[cur])
        else:  # fused: CSR edges → one-hot MFMA products, no tile
            LI.bond_fused(vb, sigma, omega, 0, members=members, agent_exposure=exposure[cur])

    def step():
        cur = it[0] & 1
        it[0] += 1
        main = torch.cuda.current_stream(ctx.dev) if side is not None else None
        if side is not None:
            side.wait_stream(main)
            with torch.cuda.stream(side):
                liability_stage(cur)
        stats.zero_()
        agents = torch.randint(0, A_, (S,), device=ctx.dev, dtype=i32, generator=gen)
        eng.run_pipeline(S, agents=agents, stats=stats)
        if side is None:
            liability_stage(cur)
        else:
            main.wait_stream(side)
        comm[cur].launch(exchange, exposure[cur])  # X01 over RCCL / xGMI, overlapped
        X.allreduce_stats(stats)

    el, lat = ctx.timed(step, args.steps, args.warmup)
    ctx.emit(config="config3", liability="tiles" if args.tiles else "fused",
             what="pipeline+sigma_eff/exposure+" + ("reduce_scatter to owners" if owner_reduce
                                                                          else "all_reduce[A]") + " (overlapped)",
             agents=A_,
             sessions_global=args.sessions or 100_000, sessions_per_rank=S, exposure_bytes=A_ * 8,
             batch_p50_ms=statistics.median(lat) * 1e3, ms_per_step=el / args.steps * 1e3,
             sessions_per_s=(args.sessions or 100_000) * args.steps / el, scaling="strong",
             parallelism=f"dp{ctx.world}")


# ------------------------------------------------------------------ config 4


def config4(ctx: Ctx, args):
    S = args.sessions or 1_000_000
    K = 10
    o = SagaOutcomes.synthetic(S, K, p_fail=0.03, p_comp_fail=0.05, p_no_undo=0.05, max_retries=1,
                               seed=ctx.rank).to(ctx.dev)
    fused = SagaBatchEngine(S, K, device=str(ctx.dev))
    el, lat = ctx.timed(lambda: fused.run(o, now_us=1), args.steps, args.warmup)
    st = fused.stats.cpu().tolist()
    ctx.emit(config="config4", mode="fused", sagas=S, steps_per_saga=K, ms_per_batch=el / args.steps * 1e3,
             batch_p50_ms=statistics.median(lat) * 1e3, sagas_per_s=S * ctx.world * args.steps / el,
             completed=st[0], escalated=st[1], compensated_steps=st[3])
    loop = SagaBatchEngine(S, K, device=str(ctx.dev))
    loop.run_step_loop(o, now_us=1)
    el, lat = ctx.timed(loop.replay if ctx.dev.type == "cuda" else (lambda: loop.run_step_loop(o, now_us=1)),
                        args.steps, args.warmup)
    ctx.emit(config="config4", mode="hipgraph_step_loop", launches_per_batch=2 * K + 3, sagas=S,
             ms_per_batch=el / args.steps * 1e3, batch_p50_ms=statistics.median(lat) * 1e3,
             sagas_per_s=S * ctx.world * args.steps / el)
    # real (stub) coroutines: SagaOrchestrator.execute_sagas awaits every executor /
    # compensator on the host (asyncio) and replays the captured step loop on the
    # device over the gathered outcomes (agent_hypervisor_amd.models.saga_runner)
    import asyncio
    import random as _random

    from hypervisor.saga.orchestrator import SagaOrchestrator

    Sc = min(S, args.coroutine_sagas)
    rng = _random.Random(ctx.rank)

    def build():
        orch = SagaOrchestrator()
        orch.DEFAULT_RETRY_DELAY_SECONDS = 0.0
        ids, ex = [], {}
        for i in range(Sc):
            sg = orch.create_saga(f"session-{i}")
            ids.append(sg.saga_id)
            for k in range(K):
                st = orch.add_step(sg.saga_id, f"a{k}", "did:mesh:agent", "/exec",
                                   "/undo" if rng.random() >= 0.05 else None, max_retries=1)
                fail = rng.random() < 0.03

                async def run(fail=fail):
                    if fail:
                        raise RuntimeError("executor failed")
                    return True

                ex[st.step_id] = run
        return orch, ids, ex

    async def compensator(step):
        return True

    times = []
    for _ in range(args.warmup + args.steps):
        orch, ids, ex = build()
        t0 = time.perf_counter()
        asyncio.run(orch.execute_sagas(ids, ex, compensator, device=str(ctx.dev)))
        ctx.sync()
        times.append(time.perf_counter() - t0)
    el = sum(times[args.warmup:])
    orch, ids, ex = build()  # the host orchestrator on the same workload, for reference
    t0 = time.perf_counter()
    asyncio.run(orch.execute_sagas(ids, ex, compensator))
    host_ms = (time.perf_counter() - t0) * 1e3
    from agent_hypervisor_amd.models.saga_runner import runner_for

    st = runner_for(ctx.dev).last_stats
    ctx.emit(config="config4", mode="coroutines+device_fsm_graph", sagas=Sc, steps_per_saga=K,
             ms_per_batch=el / args.steps * 1e3, sagas_per_s=Sc * ctx.world * args.steps / el,
             completed=st[0], escalated=st[1], compensated_steps=st[3], host_orchestrator_ms=host_ms,
             note="outcomes from awaited stub coroutines (3% failing executors, 5% steps without Undo_API)")


# ------------------------------------------------------------------ config 5


class AuditArena:
    """Resident audit chains of ``S`` sessions with distinct payloads (config 5).

    A template chain — D deltas captured through the scalar DeltaEngine, plus one
    "slash" delta whose content hash is a 256-character placeholder — is stamped
    per session on the device: session index digits into the DID, session id,
    paths and content hashes, per-session microseconds into the timestamps.
    Deltas 0..D-1 of every session live in one HBM arena; each session also owns
    a slash-delta slot in a tail region, rendered after the slash (one
    ``render_rows`` launch: template + stamps + the hex of the session's
    post-slash score row), so the re-chain depends on the slash.  The per-delta
    (prefix, suffix) spans of every session's chain are a resident table: the
    re-chain's arguments for the touched sessions are four row gathers."""

    PH, MICRO, HEXPH = b"@@@@@@@", b"999999", b"x" * 256

    def __init__(self, S: int, D: int, dev) -> None:
        from datetime import datetime, timezone

        from hypervisor import _clock
        from hypervisor.audit.delta import DeltaEngine, VFSChange

        prev = _clock._override
        _clock.set_clock(lambda: datetime(2026, 3, 1, 12, 0, 0, 999999, tzinfo=timezone.utc))
        try:
            de = DeltaEngine("session:@@@@@@@")
            for k in range(D):
                de.capture("did:mesh:agent-@@@@@@@", [VFSChange(f"/s@@@@@@@/f{k}", "add", f"h{k}-@@@@@@@")])
            de.capture("did:mesh:agent-@@@@@@@", [VFSChange("/s@@@@@@@/slash", "modify", "x" * 256)])
        finally:
            _clock.set_clock(prev)
        chain = A.pack_chains([de.deltas[:D]])
        last = A.pack_chains([de.deltas[D:]])
        self.S, self.D, self.dev = S, D, dev
        tb, lb = bytes(chain["bytes"].tolist()), bytes(last["bytes"].tolist())
        self.L, self.Ls = len(tb), len(lb)
        find = lambda buf, pat: [i for i in range(len(buf) - len(pat) + 1) if buf[i:i + len(pat)] == pat]  # noqa: E731
        self.ph, self.micro = find(tb, self.PH), find(tb, self.MICRO)
        self.s_ph, self.s_micro, self.s_hex = find(lb, self.PH), find(lb, self.MICRO), find(lb, self.HEXPH)
        assert len(self.s_hex) == 1 and self.ph and self.micro
        # resident arena: S chains, then one slash-delta slot per session (slots
        # 16-byte aligned so the render kernel writes whole words)
        self.tail = (S * self.L + 255) // 256 * 256
        self.pitch = (self.Ls + 15) // 16 * 16
        self.bytes = torch.empty(self.tail + S * self.pitch, dtype=u8, device=dev)
        body = self.bytes[: S * self.L].view(S, self.L)
        body.copy_(torch.frombuffer(bytearray(tb), dtype=u8).to(dev).expand(S, self.L))
        self._tmpl_slash = torch.frombuffer(bytearray(lb), dtype=u8).to(dev)
        idx = torch.arange(S, device=dev)
        self._stamp(body, idx, self.ph, self.micro)
        # resident span table [S, D+1]: deltas 0..D-1 in the body row, D in the slash slot
        s64 = idx.to(i64)[:, None]
        cat = lambda x, y: torch.cat([x, y], dim=1).contiguous()  # noqa: E731
        col = lambda v, dt: torch.full((S, 1), v, dtype=dt, device=dev)  # noqa: E731
        slot = self.tail + s64 * self.pitch
        self.pre_off = cat(s64 * self.L + chain["pre_off"].to(dev)[None, :], slot + int(last["pre_off"][0]))
        self.suf_off = cat(s64 * self.L + chain["suf_off"].to(dev)[None, :], slot + int(last["suf_off"][0]))
        self.pre_len = cat(chain["pre_len"].to(dev)[None, :].expand(S, D), col(int(last["pre_len"][0]), i32))
        self.suf_len = cat(chain["suf_len"].to(dev)[None, :].expand(S, D), col(int(last["suf_len"][0]), i32))
        self.chain_offsets = (torch.arange(S + 1, device=dev, dtype=i64) * (D + 1)).to(i32)

    @staticmethod
    def _digits(idx: torch.Tensor, n: int) -> torch.Tensor:
        p = 10 ** torch.arange(n - 1, -1, -1, device=idx.device)
        return ((idx[:, None] // p) % 10 + 48).to(u8)

    def _stamp(self, rows: torch.Tensor, idx: torch.Tensor, ph, micro) -> None:
        # microseconds 1..999999: a zero field would drop out of isoformat()
        d7, d6 = self._digits(idx, 7), self._digits(idx % 999_999 + 1, 6)
        for p in ph:
            rows[:, p:p + 7] = d7
        for p in micro:
            rows[:, p:p + 6] = d6

    def write_slash_deltas(self, touched: torch.Tensor, scores: torch.Tensor) -> None:
        """Slash delta of each touched session (its tail slot): the template
        stamped with the session, content hash = hex of its post-slash score row
        (row ``touched[r]`` of ``scores`` [S, 16]).  ``touched`` ⊂ [0, S)."""
        A.render_rows(self.bytes[self.tail:], self._tmpl_slash, touched.to(i64),
                      stamps=[(p, 7, 0, 0) for p in self.s_ph] + [(p, 6, 999_999, 1) for p in self.s_micro],
                      hex_field=(self.s_hex[0], scores, 128), check=False, pitch=self.pitch)

    def packed(self, touched: torch.Tensor) -> dict:
        """chain_hash arguments for the touched sessions' chains (D + 1 deltas),
        gathered from the resident span table (tests / the host path)."""
        T = touched.numel()
        g = lambda t: t.index_select(0, touched).reshape(-1)  # noqa: E731
        return {
            "bytes": self.bytes,
            "chain_offsets": self.chain_offsets[: T + 1],
            "pre_off": g(self.pre_off), "pre_len": g(self.pre_len),
            "suf_off": g(self.suf_off), "suf_len": g(self.suf_len),
        }

    def resident(self, touched: torch.Tensor) -> tuple[dict, torch.Tensor]:
        """(chain_hash arguments over the resident span table, sel): the kernels
        read chain c's spans at row touched[c] — no per-storm gather."""
        T = touched.numel()
        flat = lambda t: t.reshape(-1)  # noqa: E731
        return {
            "bytes": self.bytes,
            "chain_offsets": self.chain_offsets[: T + 1],
            "pre_off": flat(self.pre_off), "pre_len": flat(self.pre_len),
            "suf_off": flat(self.suf_off), "suf_len": flat(self.suf_len),
        }, touched


def storm_counts(out, released: torch.Tensor) -> torch.Tensor:
    """[bond updates by slash clips, bond updates by the session release] as one
    device int64 pair (no host sync): every clip releases its bond (the reference
    ``SlashingEngine.slash`` calls ``release_bond`` per clip, slashing.py:93-112),
    and K07 releases each session's remaining active bonds
    (``release_session_bonds``, vouching.py:176-184)."""
    return torch.stack([out.clip_count.sum(dtype=i64), released.sum(dtype=i64)])


def config5(ctx: Ctx, args):
    """BASELINE config 5 as stated: "Liability slash storm: 10M bond updates + full
    Merkle re-chain".  Every session is slashed (storm fraction 1.0: one vouchee per
    session, cascades included) and then has its remaining bonds released, so every
    one of the 10M resident edges changes state; every session gets its slash delta
    and its WHOLE chain is re-hashed and Merkle-rooted.  The bond-update count is
    the device's (clip counts + K07 release counts), not the resident edge count.
    ``--storm-fraction f < 1`` gives the secondary storm over a session subset with
    only the touched sessions re-chained (the round-5 measurement)."""
    frac = args.storm_fraction
    _storm(ctx, args, frac, rechain_all=frac >= 1.0, release_all=frac >= 1.0)


def _storm(ctx: Ctx, args, frac: float, rechain_all: bool, release_all: bool):
    E_total = args.edges or 10_000_000
    per = 16
    S = E_total // per
    vb0 = random_vouch_batch(S, per, ctx.dev, seed=5)
    g = torch.Generator().manual_seed(9)
    # the storm hits a random subset of the sessions (all of them at fraction 1.0);
    # the others keep target 255 (no slash)
    tgt = torch.full((S,), 255, dtype=u8)
    hit = torch.randperm(S, generator=g)[: max(1, int(round(S * frac)))]
    tgt[hit] = torch.randint(0, 16, (hit.numel(),), generator=g, dtype=u8)
    tgt = tgt.to(ctx.dev)
    omega = torch.full((S,), 0.95, dtype=f64, device=ctx.dev)
    scores0 = torch.rand((S, 16), generator=g, dtype=f64).to(ctx.dev)
    D = args.deltas or 3
    arena = AuditArena(S, D, ctx.dev)
    every = torch.arange(S, dtype=i64, device=ctx.dev)
    last = {}
    # Every storm starts from the same resident state.  The slash mutates only
    # `active`, `released_us` and the scores, so one fresh copy of those per storm
    # is made up front (setup, outside the timed region: ~170 MB each).
    runs = args.warmup + max(3, min(10, args.steps)) + args.steps
    fresh = [(vb0.active.clone(), vb0.released_us.clone(), scores0.clone()) for _ in range(runs)]
    # K07 (memory bound: the bond columns) on a side stream beside the re-chain's SHA
    # passes (VALU bound), which read nothing it writes; --serial-release: in line
    side = torch.cuda.Stream(ctx.dev) if ctx.dev.type == "cuda" and release_all and not args.serial_release else None

    def step():
        active, released, scores = fresh.pop()
        vb = LI.VouchBatch(vb0.offsets, vb0.voucher, vb0.vouchee, vb0.bonded, active, vb0.expiry_us, released)
        # ≤ 1 clip per edge; σ_eff over the post-slash bonds fused into the same pass (K06+K03)
        out = LI.slash(vb, tgt, omega, scores, 1, clip_cap=per, zero_records=False, with_sigma_eff=not args.unfused,
                       with_touched=not rechain_all)
        se = out.sigma_eff if not args.unfused else LI.sigma_eff_exact(vb, out.scores, omega, 1)
        rel = None
        if release_all and side is not None:  # K07: the storm's sessions end — every bond still active is released
            side.wait_stream(torch.cuda.current_stream(ctx.dev))  # after the slash's clips
            with torch.cuda.stream(side):
                rel = LI.release_bonds(vb, 2)
        elif release_all:
            rel = LI.release_bonds(vb, 2)
        else:
            rel = torch.zeros(1, dtype=i32, device=ctx.dev)
        # re-chain after the slash (data dependency): each session gets a slash delta
        # carrying its post-slash scores, then its whole chain is re-hashed (K08) and
        # its Merkle root recomputed (K09) — every session, or (subset storm) the ones
        # the slash touched, compacted on the device (one 8-byte count read)
        touched = every if rechain_all else out.touched
        arena.write_slash_deltas(touched, out.scores)
        packed, sel = arena.resident(touched)
        digests = A.chain_hashes(packed, midstate=not args.no_midstate, uniform_len=D + 1, sel=sel, check=False)
        roots = A.merkle_roots(packed["chain_offsets"], digests)
        if side is not None:  # the release joins before the storm ends
            torch.cuda.current_stream(ctx.dev).wait_stream(side)
            rel.record_stream(torch.cuda.current_stream(ctx.dev))
        last["counts"] = storm_counts(out, rel)
        last.update(T=touched.numel(), roots=roots)
        return se

    el, lat = ctx.timed(step, args.steps, args.warmup)
    T = int(last["T"])
    by_slash, by_release = (int(x) for x in last["counts"].cpu().tolist())
    updates = by_slash + by_release
    ms = el / args.steps * 1e3
    # HBM traffic per storm (bytes, lower bound: each array touched once)
    slash_bytes = S * per * (1 + 1 + 2 + 8 + 8 + 8) + S * 16 * 8 * 2 + S * 16 * 8 + S * 4
    release_bytes = (S * per * (2 + 8 + 8) + S * 8) if release_all else 0
    rechain_bytes = T * (arena.L + 2 * arena.pitch) + T * (D + 1) * 32 * 2 + T * 32 + T * 16 * 8
    hbm = slash_bytes + release_bytes + rechain_bytes
    # SHA-256 compressions on the re-chain path (records + Merkle nodes)
    blocks_per_chain = int(sum((int(x) + 9 + 63) // 64 for x in (arena.pre_len[0] + arena.suf_len[0]).tolist())) \
        + 2 * max(1, D)  # ~2 blocks per Merkle node (hex-pair message), D nodes for D+1 leaves
    ctx.emit(config="config5" if rechain_all else "config5_subset",
             what=("slash storm over every session (all bonds clipped or released) + sigma_eff + full re-chain/"
                   "Merkle of every session" if rechain_all else
                   "slash storm on a session subset + sigma_eff + re-chain/merkle of the touched sessions"),
             bond_edges_resident=S * per, sessions=S, storm_fraction=frac,
             sessions_slashed=int(hit.numel()), bond_updates=updates, bond_updates_by_slash=by_slash,
             bond_updates_by_release=by_release, sessions_rechained=T, deltas_rechained=T * (D + 1),
             arena_bytes_resident=int(arena.bytes.numel()), distinct_payloads=True,
             state_reset="one pre-made copy of (active, released_us, scores) per storm, made before timing",
             release_stream="side (beside the re-chain)" if side is not None else "main",
             hbm_bytes_est=dict(slash_sigma=slash_bytes, release=release_bytes, rechain=rechain_bytes, total=hbm),
             hbm_roofline_ms=round(hbm / 8.0e12 * 1e3, 4), hbm_achieved_tb_s=round(hbm / (ms * 1e-3) / 1e12, 3),
             sha_compressions_est=T * blocks_per_chain,
             ms_per_storm=ms, storm_p50_ms=statistics.median(lat) * 1e3,
             bond_updates_per_s=updates * ctx.world / (ms * 1e-3),
             sessions_rechained_per_s=T * ctx.world / (ms * 1e-3))


def config5_subset(ctx: Ctx, args):
    """Secondary config-5 line: the storm over ``--subset-fraction`` (10 %) of the
    sessions, only the touched sessions re-chained (no session release)."""
    _storm(ctx, args, args.subset_fraction, rechain_all=False, release_all=False)


# ------------------------------------------------------------------ config 2 (public API)


def config2_api(ctx: Ctx, args):
    """BASELINE config 2 through the public API: 10⁴–10⁵ concurrent sessions, each
    a full governance pipeline (joins with σ ring gates, audit deltas, saga steps,
    terminate with its Merkle root committed) written into the device store by
    ``Hypervisor.run_pipelines`` — once with the reference template, once with a
    randomized spec per session (heterogeneous) — and the per-call pipeline under
    ``asyncio.gather`` for comparison (benchmarks/bench_api.py)."""
    from benchmarks.bench_api import api_throughput, batch_api_throughput

    n = args.sessions or 100_000
    dev = str(ctx.dev)
    t = batch_api_throughput(dev, n, max(1, args.steps // 3))
    h = batch_api_throughput(dev, n, max(1, args.steps // 5), hetero=True)
    g = api_throughput(dev, min(n, 10_000), 1)
    ctx.emit(config="config2_api", what="public API: batched store pipelines (template / heterogeneous) and "
                                        "per-call asyncio.gather", sessions=n,
             template_sessions_per_s=t["sessions_per_s"], template_device_ms=t["device_ms"],
             hetero_sessions_per_s=h["sessions_per_s"], hetero_device_ms=h["device_ms"],
             gather_pipelines_per_s=g["pipelines_per_s"], gather_concurrent=g["concurrent_pipelines"],
             ok=bool(t["ok"] and h["ok"] and g["roots_ok"]))


def main():
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("configs", nargs="*", default=["config2", "config3", "config4", "config5", "config5_subset"])
    ap.add_argument("--device", choices=("cuda", "cpu"), default="cuda")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--sessions", type=int, default=0, help="override the config's session/saga count")
    ap.add_argument("--agents", type=int, default=0)
    ap.add_argument("--edges", type=int, default=0)
    ap.add_argument("--deltas", type=int, default=0)
    ap.add_argument("--storm-fraction", type=float, default=1.0,
                    help="config5: share of sessions slashed (1.0: BASELINE config 5 as stated)")
    ap.add_argument("--subset-fraction", type=float, default=0.1, help="config5_subset: share of sessions slashed")
    ap.add_argument("--coroutine-sagas", type=int, default=4096, help="config4: sagas in the coroutine mode")
    ap.add_argument("--unfused", action="store_true", help="config5: separate slash and sigma_eff passes (A/B)")
    ap.add_argument("--unfused-graph", action="store_true",
                    help="config2: separate zero/clock/fold/advance graph nodes instead of the fused epilogue (A/B)")
    ap.add_argument("--no-midstate", action="store_true", help="config5: single-phase K08 re-chain (A/B)")
    ap.add_argument("--serial-release", action="store_true",
                    help="config5: K07 in line on the main stream, not beside the re-chain (A/B)")
    ap.add_argument("--tiles", action="store_true", help="config3: round-1 build_tiles + bond_tiles pair")
    ap.add_argument("--allreduce-exposure", action="store_true",
                    help="config3: all-reduce the full exposure vector on every rank instead of the default "
                         "reduce-scatter to agent owners (P02)")
    args = ap.parse_args()
    ctx = Ctx(args.device)
    for c in args.configs:
        {"config2": config2, "config2_api": config2_api, "config3": config3, "config4": config4,
         "config5": config5, "config5_subset": config5_subset}[c](ctx, args)
    if ctx.world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
