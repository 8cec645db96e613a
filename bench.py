#!/usr/bin/env python3
"""Headline benchmark: the reference's ``full_governance_pipeline`` on MI355X.

BASELINE.json metric: "p50 pipeline latency (µs) + session-ops/sec,
bench_hypervisor.py at 1/2/4/8 GPU".  One *session-op* is one complete run of the
reference pipeline (bench_hypervisor.py:217-239) for one session: create → join
(σ ring gate) → activate → 3 audit deltas (canonical JSON + SHA-256 Merkle chain)
→ saga create/add/execute step → terminate (Merkle root, commitment, bond
release, GC, archive).

Each timed step runs that pipeline for ``--sessions`` new sessions per GPU in one
gfx950 launch over the device store's rows (``store_template_kernel``: session,
participant, delta rows with their canonical-JSON records in the payload arena,
saga and step rows — the same rows the per-call API writes, so every session is
an ordinary store session; rows allocated once and freed in place every step;
device-minted ids, synthetic agents with random-init σ), then a cross-rank RCCL
all-reduce of the step's governance counters (collective X04) — weak scaling,
sessions sharded data-parallel.  (``--graph`` replays the older standalone
engine-table kernel from a captured hipGraph.)

Cross-session liability propagation runs inside the same timed step, on a side
stream overlapping the pipeline kernel (``--no-liability`` turns it off): over a
resident bond graph of ``--agents`` agents × ``--bond-degree`` edges per rank,
the K04 exposure partial → X01 all-reduce of the [A] fp64 agent-exposure vector
(8 MB at 1 M agents) over xGMI, and a K06 slash stage of ``--slash-k`` vouchees
→ X02 sparse merge (fixed-capacity (agent, factor) all-gather + PROD scatter)
into the agent σ vector.  Bytes per step of every collective are in the JSON.

Also reported (not the headline value):
* ``device_p50_us`` — p50 of the single-session pipeline through the public
  ``Hypervisor(device="cuda")`` API, reference harness methodology (2,000
  iterations after warm-up): every state change, ring gate, audit digest,
  Merkle root, bond release and saga transition is executed by the resident
  gfx950 store worker (hypervisor/_device.py, csrc/hip/store_worker.hip), and
  terminate returns the Merkle root the device computed (awaited);
* ``device_p50_speculated_us`` — the same with ``AHV_SPEC_TERMINATE=1``: terminate
  returns the host's SHA-NI prediction of the root at once and the device's
  committed root is checked afterwards (a divergence poisons the session);
* ``scalar_p50_us`` — the same harness on the pure host engines (CPU only);
* ``batch_p50_ms`` — p50 wall time of one synchronised pipeline step;
* ``api`` — public-API throughput after the timed region (rank 0, 1 GPU runs),
  in reference pipelines per second: the batched API ``Hypervisor.run_pipelines``
  over 10⁵ pipelines written into the device store (wall clock incl. host-side
  registration), a randomized-spec batch, and 10⁴ concurrent per-call pipelines
  under ``asyncio.gather`` on the device and on the host engines (``--no-api``
  skips).

``vs_baseline`` divides the batched GPU throughput by the reference's
single-threaded Python pipeline rate — a capability ratio, not a like-for-like
one; ``device_vs_baseline_p50`` compares like with like (one session, public
API, same harness).

Launch: ``python bench.py`` (1 GPU); ``python bench.py --gpus N`` starts N rank
processes itself (one per GPU, RCCL over xGMI; see :func:`launch_ranks`), and under
``torch.distributed.run`` the launcher's ``WORLD_SIZE`` must equal ``--gpus``.
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


def scalar_pipeline_p50(iters: int = 2000, device: str = "host", speculate: bool = False) -> tuple[float, float]:
    """Reference-harness timing of the public-API pipeline (bench_hypervisor.py:217-239).

    ``device="host"``: pure host engines; ``device="cuda"``: the device-authoritative
    store (every call is a command to the gfx950 worker; terminate returns the root
    the device computed).  ``speculate``: terminate returns the host's prediction of
    the root at once and the device's answer is checked afterwards."""
    from hypervisor import Hypervisor, SessionConfig
    from hypervisor import _device as D
    from hypervisor.audit.delta import VFSChange

    D._SPEC_TERMINATE = speculate

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

    try:
        times = asyncio.run(run())
    finally:
        D._SPEC_TERMINATE = os.environ.get("AHV_SPEC_TERMINATE", "0") != "0"
    return statistics.median(times) / 1000.0, statistics.mean(times) / 1000.0


def api_section(args, scalar_p50) -> dict:
    """Public-API throughput on this GPU (outside the timed step; rank 0).

    * ``batch``: :meth:`Hypervisor.run_pipelines` — ``--api-sessions`` reference
      pipelines per call through the public batched API, written into the device
      store and registered as ordinary sessions (median of 3 calls, a fresh
      Hypervisor each, wall clock incl. registration and teardown);
    * ``batch_hetero``: the same with a randomized spec per session;
    * ``gather``: ``--api-concurrent`` per-call pipelines under one asyncio.gather
      through ``Hypervisor(device="cuda")`` (reference bench_hypervisor.py:217-239),
      and the same harness on the host engines.
    All rates are whole reference pipelines per second."""
    from benchmarks.bench_api import api_throughput, batch_api_throughput

    b = batch_api_throughput("cuda", args.api_sessions, 3)
    bh = batch_api_throughput("cuda", max(1, args.api_sessions // 5), 2, hetero=True)
    g = api_throughput("cuda", args.api_concurrent, 1)
    h = api_throughput("host", args.api_concurrent, 1)
    host_scalar = 1e6 / scalar_p50 if scalar_p50 else None
    rate = b["sessions_per_s"]
    return {
        "batch_pipelines_per_s": rate, "batch_sessions": args.api_sessions, "batch_ok": b["ok"],
        "batch_device_ms": b["device_ms"],
        "batch_hetero_sessions_per_s": bh["sessions_per_s"], "batch_hetero_sessions": bh["sessions"],
        "gather_pipelines_per_s": g["pipelines_per_s"], "gather_concurrent": args.api_concurrent,
        "host_gather_pipelines_per_s": h["pipelines_per_s"],
        "host_scalar_pipelines_per_s": round(host_scalar, 1) if host_scalar else None,
        "batch_vs_host_scalar": round(rate / host_scalar, 2) if host_scalar else None,
        "batch_vs_host_gather": round(rate / h["pipelines_per_s"], 2),
    }


def _headline_kernel(n: int) -> str:
    """The store_template_kernel variant a batch of ``n`` sessions runs (store_template.hip)."""
    if n <= int(os.environ.get("AHV_TEMPLATE_SMALL", "65536")):
        return "store_template_kernel<1,6>"
    w = int(os.environ.get("AHV_TEMPLATE_WAVES", "3"))
    return {2: "store_template_kernel<2,3>", 4: "store_template_kernel<4,2>"}.get(w, "store_template_kernel<3,3>")


def _free_port() -> int:
    import socket

    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(n: int, argv: list[str], grace_s: float = 30.0) -> int:
    """``bench.py --gpus N`` without a launcher: start N rank processes (one per GPU).

    Runs in the parent BEFORE any GPU call (``torch.cuda.device_count()`` does not
    initialise HIP on this image, nothing else here touches the device), and starts
    every rank as a fresh child — the parent is never re-executed.  Each child gets
    RANK / LOCAL_RANK / WORLD_SIZE / LOCAL_WORLD_SIZE / MASTER_ADDR / MASTER_PORT as
    ``torch.distributed.run`` would set them, inherits stdout (rank 0 prints the one
    JSON line) and stderr.  If a rank fails, the others get ``grace_s`` to finish and
    are then terminated (a peer blocked in a collective would otherwise wait for
    ever).  Returns the worst exit code over the ranks (0 iff every rank succeeded).

    The reference harness is single-process (bench_hypervisor.py:246-304); the
    multi-rank launch is this framework's own (weak scaling, one process per GPU)."""
    import subprocess

    port = int(os.environ.get("MASTER_PORT") or _free_port())
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR=os.environ.get("MASTER_ADDR", "127.0.0.1"), MASTER_PORT=str(port),
                   AHV_BENCH_SPAWNED="1")
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__), *argv], env=env, cwd=ROOT))
    codes: dict[int, int] = {}
    failed_at = None
    while len(codes) < n:
        for r, p in enumerate(procs):
            if r not in codes and p.poll() is not None:
                codes[r] = p.returncode
                if p.returncode != 0 and failed_at is None:
                    failed_at = time.monotonic()
                    print(f"bench.py: rank {r} exited with {p.returncode}", file=sys.stderr, flush=True)
        if failed_at is not None and time.monotonic() - failed_at > grace_s:
            for r, p in enumerate(procs):
                if r not in codes:
                    p.terminate()
                    try:
                        codes[r] = p.wait(10)
                    except subprocess.TimeoutExpired:
                        p.kill()
                        codes[r] = p.wait()
        time.sleep(0.05)
    bad = [c for c in codes.values() if c != 0]
    return (max(bad, key=abs) if bad else 0)


def main() -> None:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--verify-sessions", type=int, default=64,
                    help="sessions of the last timed step oracle-checked against the host after timing")
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--sessions", type=int, default=1 << 22,
                    help="sessions per GPU per step (4M: the launch amortises its tail; 1M measured 7%% lower)")
    ap.add_argument("--agents", type=int, default=1 << 20, help="synthetic agents per GPU")
    ap.add_argument("--deltas", type=int, default=3)
    ap.add_argument("--scalar-iters", type=int, default=2000)
    ap.add_argument("--no-scalar", action="store_true")
    ap.add_argument("--no-api", action="store_true", help="skip the public-API throughput section")
    ap.add_argument("--api-sessions", type=int, default=100_000, help="sessions per batched API call")
    ap.add_argument("--api-concurrent", type=int, default=10_000, help="concurrent per-call pipelines (gather)")
    ap.add_argument("--graph", action="store_true",
                    help="replay each step from a captured hipGraph (device cursor + RCCL counters)")
    ap.add_argument("--no-liability", action="store_true", help="skip the X01/X02 liability stage")
    ap.add_argument("--join-liability", action="store_true",
                    help="join the liability side stream with the pipeline stream every step (A/B)")
    ap.add_argument("--bond-degree", type=int, default=4, help="resident vouch edges per agent")
    ap.add_argument("--slash-k", type=int, default=1024, help="vouchees slashed per step (X02 stage)")
    ap.add_argument("--mix", choices=("template", "hetero"), default="template",
                    help="template: the reference pipeline for every session (headline kernel); hetero: a "
                         "heterogeneous mix (store_pipeline.mixed_specs) through the public batched API's kernels "
                         "over store rows (rows / render / chain + K09 roots, rows freed and rebuilt every step)")
    ap.add_argument("--participant-rows", type=int, default=16,
                    help="participant rows per session row of the headline store (SessionConfig.max_participants "
                         "of the template is 10; a join past the row width is refused)")
    ap.add_argument("--device", choices=("cuda", "cpu"), default="cuda",
                    help="cpu runs the host twin of the kernel over gloo (multi-process CPU rehearsal)")
    args = ap.parse_args()

    if args.gpus < 1:
        raise SystemExit("bench.py: --gpus must be >= 1")
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # No launcher around us: start the N ranks ourselves (fresh children, before any
        # GPU call in this process) and exit with the worst rank's code.
        if args.device == "cuda" and torch.cuda.device_count() < args.gpus:
            raise SystemExit(f"bench.py: --gpus {args.gpus} but only {torch.cuda.device_count()} GPUs are visible")
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        # under a launcher the job's world size IS the GPU count the run reports
        raise SystemExit(f"bench.py: WORLD_SIZE={world} but --gpus {args.gpus}; the run would not measure N GPUs")
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
            # RCCL's internal streams at high priority: the collectives' workgroups are
            # dispatched ahead of the pipeline kernel's queued waves instead of behind them
            opts = dist.ProcessGroupNCCL.Options()
            opts.is_high_priority_stream = True
            dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev, pg_options=opts)
        else:
            dist.init_process_group("gloo", rank=rank, world_size=world)

    def sync():
        if dev.type == "cuda":
            torch.cuda.synchronize(dev)

    from agent_hypervisor_amd.parallel.collectives import allreduce_stats  # noqa: F401 (graph mode)

    S = args.sessions
    g = torch.Generator(device=dev).manual_seed(77 + rank)
    tmpl = None
    eng = None
    if args.graph:
        from agent_hypervisor_amd.models.engine import GovernanceEngine

        eng = GovernanceEngine(
            device=str(dev), session_capacity=2 * S, agent_capacity=args.agents, seed=0x5EED0000 + rank
        )
        eng.register_synthetic_agents(args.agents, seed=1000 + rank, prefix=f"did:mesh:r{rank}-agent-")
    elif args.mix == "template":
        # The headline step writes the device store's rows (one device state): the
        # template pipeline kernel over rows allocated once and freed in place every
        # step — every session is an ordinary store session (session, participant,
        # delta rows + canonical-JSON records in the payload arena, saga and step rows).
        from agent_hypervisor_amd.models import store_template as TT
        from agent_hypervisor_amd.models.store import GovernanceStore

        nd = max(1, S * args.deltas)
        caps = {"S": S, "G": S, "T": S, "D": nd, "P": args.participant_rows, "E": 1 << 12, "V": 1 << 12, "X": 1 << 22,
                "B": nd * 384 + (1 << 20)}
        tstore = GovernanceStore(str(dev), caps=caps, max_caps={k: v for k, v in caps.items() if k not in ("P", "X")})
        tagents = TT.AgentSet.synthetic(tstore, args.agents, seed=1000 + rank, prefix=f"did:mesh:r{rank}-agent-")
        tmpl = TT.TemplatePipeline(tstore, S, tagents, deltas=args.deltas, seed=0x5EED0000 + rank)
        first = torch.randint(0, args.agents, (S,), device=dev, dtype=torch.int32, generator=g)
        tmpl.launch(first, sync=True)  # first run over the freshly allocated rows (checks them)
        if not bool((tmpl.tens["status"] == 0).all()):
            raise SystemExit("template pipeline: rows refused on the first run")
    stats = torch.zeros(6, dtype=torch.int64, device=dev)

    # X04 counters: double-buffered so step i's all-reduce (RCCL, on its own
    # stream) overlaps step i+1's pipeline kernel; a buffer is reused only after
    # its collective from two steps back has completed (a stream wait, no host sync).
    bufs = [torch.zeros(6, dtype=torch.int64, device=dev) for _ in range(2)]
    works: list = [None, None]
    it = [0]

    # Liability stage (X01/X02) on a side stream: resident bonds, exposure, slash storm.
    liab = None
    if not args.no_liability:
        from agent_hypervisor_amd.ops.global_liability import ResidentBonds
        from agent_hypervisor_amd.parallel.collectives import merge_slash_fixed

        A = args.agents
        bonds = ResidentBonds(A, args.bond_degree, dev, seed=4242 + rank)
        k = args.slash_k
        cap = 16 * k
        liab = {
            "bonds": bonds,
            "expo": torch.zeros(A, dtype=torch.float64, device=dev),
            "sigma": torch.rand(A, dtype=torch.float64, device=dev, generator=g),
            "ids": torch.zeros(k, dtype=torch.int32, device=dev),
            "pid": torch.full((cap,), -1, dtype=torch.int32, device=dev),
            "pf": torch.ones(cap, dtype=torch.float64, device=dev),
            "cur": torch.zeros(1, dtype=torch.int64, device=dev),
            "factor": torch.ones(A, dtype=torch.float64, device=dev),
            "work": None,
            "stream": torch.cuda.Stream(dev, priority=-1) if dev.type == "cuda" else None,
            "gen": torch.Generator(device=dev).manual_seed(99 + rank),
        }
        x01_bytes = A * 8
        x02_bytes = k * 4 + cap * 12  # per rank: blacklist ids (i32) + (id i32, factor f64) pairs
        if liab["stream"] is not None:  # the stage's buffers were initialised on the main stream
            liab["stream"].wait_stream(torch.cuda.current_stream(dev))

    def liability_step():
        L = liab
        if L["work"] is not None:
            L["work"].wait()  # the previous step's X01 must finish before the buffer is rewritten
        L["bonds"].exposure(L["expo"])  # K04 partial
        L["work"] = dist.all_reduce(L["expo"], op=dist.ReduceOp.SUM, async_op=True) if multi else None  # X01
        L["ids"].random_(0, args.agents, generator=L["gen"])
        L["cur"].zero_()
        L["pid"].fill_(-1)
        L["pf"].fill_(1.0)
        L["bonds"].slash_clip(L["ids"], 0.95, L["pid"], L["pf"], L["cur"])  # K06 stage
        merge_slash_fixed(L["sigma"], L["ids"], L["pid"], L["pf"], factor=L["factor"])  # X02

    hetero = None
    if args.mix == "hetero":
        # The public batched API's kernels over the device store (Hypervisor.run_pipelines):
        # the batch is packed once (host), then every step frees its session rows in place
        # and runs the whole pipeline over them again (create, joins, activate, rendered
        # and SHA-chained deltas, sagas with retries/compensation rewritten whole in the
        # batch's saga / step rows, terminate, Merkle roots).
        from agent_hypervisor_amd.models import store_pipeline as SP
        from hypervisor import Hypervisor

        os.environ.setdefault("AHV_STORE_SESSIONS", str(1 << 21))
        hv = Hypervisor(device="cuda" if dev.type == "cuda" else "cpu")
        hp = SP.prepare(hv, SP.mixed_specs(S, seed=11 + rank))
        SP.launch(hp)  # first run (also builds the K09 plan)
        status0 = hp.tens["status"].clone()
        hetero = {"hv": hv, "p": hp, "status0": status0,
                  "deltas": int(hp.nd), "committed": len(hp.committed), "ok": int((status0 == 0).sum())}

    last_launch: dict = {}

    def run_batch(st, agents):
        if tmpl is not None:
            tmpl.reset()
            last_launch["ids"] = tmpl.launch(agents, stats=st, sync=False)
            last_launch["agents"] = agents
            return
        if hetero is None:
            eng.run_pipeline(S, agents=agents, deltas=args.deltas, stats=st)
            return
        hp = hetero["p"]
        hp.reset()
        SP.launch(hp, sync=False)
        st[0] = S
        st[1] = (hp.tens["status"] == 0).sum()

    def step():
        b = it[0] & 1
        it[0] += 1
        if works[b] is not None:
            works[b].wait()
        st = bufs[b]
        side = liab["stream"] if liab is not None else None
        if side is not None:
            # The liability stage reads and writes nothing the pipeline touches, and
            # its own steps are ordered by its stream, so it runs beside the pipeline
            # with no cross-stream joins (each join is a barrier packet the main
            # queue processes between pipeline launches); the timed region's final
            # synchronize covers both streams.  --join-liability restores per-step joins.
            if args.join_liability:
                side.wait_stream(torch.cuda.current_stream(dev))
            with torch.cuda.stream(side):
                liability_step()
        st.zero_()
        # (the heterogeneous batch carries its own agents in its specs)
        agents = torch.randint(0, args.agents, (S,), device=dev, dtype=torch.int32, generator=g) \
            if hetero is None else None
        run_batch(st, agents)
        works[b] = dist.all_reduce(st, op=dist.ReduceOp.SUM, async_op=True) if multi else None
        if side is not None:
            if args.join_liability:
                torch.cuda.current_stream(dev).wait_stream(side)
        elif liab is not None:
            liability_step()
        return st

    def drain():
        for k in range(2):
            if works[k] is not None:
                works[k].wait()
                works[k] = None
        if liab is not None and liab["work"] is not None:
            liab["work"].wait()
            liab["work"] = None

    if args.graph and hetero is not None:
        raise SystemExit("--graph captures the template pipeline; --mix hetero runs on the stream")
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

        def step():  # noqa: F811 - graph-replay form of the same step (liability stage included)
            side = liab["stream"] if liab is not None else None
            if side is not None:
                with torch.cuda.stream(side):
                    liability_step()
            pg.step()
            if side is None and liab is not None:
                liability_step()
            return stats

        def drain():  # noqa: F811 - the graph's collective is in-stream; the liability X01 is not
            if liab is not None and liab["work"] is not None:
                liab["work"].wait()
                liab["work"] = None

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
    if hetero is not None:  # every re-run produced exactly the first run's per-session outcomes
        sync()
        assert torch.equal(hetero["p"].tens["status"], hetero["status0"]), "hetero batch outcomes changed between runs"
    # X09: job-wide step-latency histogram (log2 µs bins), summed over ranks outside the timed loop
    from agent_hypervisor_amd.parallel.collectives import reduce_histogram

    hist = torch.zeros(32, dtype=torch.int64)
    for x in lat:
        hist[min(31, max(0, int(x * 1e6).bit_length() - 1))] += 1
    hist = reduce_histogram(hist.to(dev)).cpu().tolist()

    scalar_p50 = scalar_mean = device_p50 = device_mean = spec_p50 = spec_mean = None
    if rank == 0 and not args.no_scalar:
        scalar_p50, scalar_mean = scalar_pipeline_p50(args.scalar_iters, "host")
        if dev.type == "cuda":
            device_p50, device_mean = scalar_pipeline_p50(args.scalar_iters, "cuda")
            spec_p50, spec_mean = scalar_pipeline_p50(args.scalar_iters, "cuda", speculate=True)

    api = None
    if rank == 0 and world == 1 and not args.no_api and dev.type == "cuda":  # 1-GPU runs (the N>1 scaling runs skip it)
        api = api_section(args, scalar_p50)

    verified = None
    if tmpl is not None:  # the rows the timed steps wrote are ordinary store sessions: oracle-check some
        sync()
        assert bool((tmpl.tens["status"] == 0).all()), "template pipeline refused sessions"
        id_base, t0 = last_launch["ids"]
        pick = torch.randint(0, S, (args.verify_sessions,), generator=torch.Generator().manual_seed(99 + rank))
        # arena records, d_hash, s_head and s_root of the last timed step vs scalar render + hashlib
        verified = TT.check_sessions(tmpl, id_base, t0, last_launch["agents"], pick.numpy())
    rccl_ranks = dist.get_world_size() if (multi and dev.type == "cuda" and dist.get_backend() == "nccl") else 0
    if dev.type == "cuda" and args.gpus > 1 and rccl_ranks != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} ran over {rccl_ranks} RCCL ranks")
    if multi and dist.get_world_size() != args.gpus:
        raise SystemExit(f"bench.py: process group has {dist.get_world_size()} ranks, --gpus {args.gpus}")
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
                "model": "full_governance_pipeline" if hetero is None else "heterogeneous_governance_pipeline",
                "global_batch": S * world,
                "seq_len": args.deltas if hetero is None else round(hetero["deltas"] / S, 3),
                "parallelism": f"dp{world}",
                "sessions_per_gpu": S,
                "agents_per_gpu": args.agents,
                "deltas_per_session": args.deltas if hetero is None else round(hetero["deltas"] / S, 3),
            },
            "batch_p50_ms": round(statistics.median(lat) * 1000.0, 4),
            "pipeline_launch": "hipgraph" if args.graph else "stream",
            "vs_baseline_note": "batched GPU throughput / single-threaded Python reference rate (not like-for-like)",
            "device_p50_us": round(device_p50, 2) if device_p50 is not None else None,
            "device_p50_speculated_us": round(spec_p50, 2) if spec_p50 is not None else None,
            "device_mean_speculated_us": round(spec_mean, 2) if spec_mean is not None else None,
            "device_mean_us": round(device_mean, 2) if device_mean is not None else None,
            "device_vs_baseline_p50": round(BASELINE_P50_US / device_p50, 3) if device_p50 else None,
            "scalar_p50_us": round(scalar_p50, 2) if scalar_p50 is not None else None,
            "scalar_mean_us": round(scalar_mean, 2) if scalar_mean is not None else None,
            "scalar_vs_baseline_p50": round(BASELINE_P50_US / scalar_p50, 2) if scalar_p50 else None,
            "api_batch_pipelines_per_s": api["batch_pipelines_per_s"] if api else None,
            "api_gather_pipelines_per_s": api["gather_pipelines_per_s"] if api else None,
            "api": api,
            "last_step_counters": dict(zip(["sessions", "ok", "participants", "deltas", "commits", "archived"],
                                           totals)),
            "step_latency_hist_log2_us": {str(1 << b): c for b, c in enumerate(hist) if c},
            "rccl_ranks": rccl_ranks,
            "launcher": "bench.py (self-spawned ranks)" if os.environ.get("AHV_BENCH_SPAWNED") == "1"
                        else ("external" if "WORLD_SIZE" in os.environ else "none (1 rank)"),
            "collective_backend": dist.get_backend() if multi else None,
            "collectives_per_step": {
                "x04_counters_bytes": 48,
                "x01_exposure_allreduce_bytes": x01_bytes if liab is not None else 0,
                "x02_slash_allgather_bytes_per_rank": x02_bytes if liab is not None else 0,
            },
            "headline_verified": bool(verified) if tmpl is not None else None,
            "headline_verified_sessions": verified,
            "headline_kernel": ((_headline_kernel(S) if dev.type == "cuda" else "host twin")
                                if tmpl is not None else None),
            "mix": args.mix,
            "state": "governance_tables (--graph)" if eng is not None else "store rows",
            "hetero": None if hetero is None else {
                "sessions": S, "deltas": hetero["deltas"], "committed_roots": hetero["committed"],
                "sessions_all_stages_admitted": hetero["ok"], "spec_pool": 4096,
                "path": "store_pipeline rows/render/chain kernels + K09 over store rows"},
            "liability_stage": None if liab is None else {
                "agents": args.agents, "resident_edges": liab["bonds"].edges, "slash_k": args.slash_k,
                "bond_graph_bytes": liab["bonds"].nbytes, "in_timed_region": True,
            },
        }
        print(json.dumps(out), flush=True)
    if multi:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
