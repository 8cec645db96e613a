"""Rank-local serving: N ranks each serving their own sessions at once do so with
zero collectives and zero forwarded messages on the per-session path (counted;
the throughput ratio is reported, not asserted) (every liability invariant is
session-scoped, so the pipeline needs no communication).

gloo on CPU, one process per rank (the same code drives RCCL on MI355X).  Each
rank runs the reference pipeline (``benchmarks/bench_hypervisor.py:217-239``)
through :class:`ShardedHypervisor` on sessions it creates.  The phases are
interleaved and repeated so machine noise hits both alike: every round runs

* **A** — rank 0 serves ``K`` pipelines while the other ranks keep their cores
  busy with a fixed CPU load that is *not* the hypervisor (so A and B run at the
  same machine load — clock boost, shared caches — and the comparison isolates
  the serving path itself), then
* **B** — every rank serves ``K`` pipelines on its own sessions at once,

and efficiency = the median over rounds of (B aggregate / (N × A rate of the same
round)): pairing each B with the A just before it cancels the host's slow drifts
(this container's vCPUs share a host).  Each rank is pinned to its own vCPU.
The idle-baseline ratio (A with the other ranks idle, one extra round) is
reported alongside; it also folds in the machine's own single-core boost.
"""

from __future__ import annotations

import asyncio
import hashlib
import os
import statistics
import time

import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

K = 400  # pipelines per rank per phase
ROUNDS = 2


async def _pipeline(shv) -> None:
    from hypervisor import SessionConfig
    from hypervisor.audit.delta import VFSChange

    sid = await shv.create_session(SessionConfig(enable_audit=True), "did:mesh:admin")
    await shv.join_session(sid, "did:mesh:a", sigma_raw=0.8)
    await shv.activate_session(sid)
    m = shv.local._get_session(sid)
    for i in range(3):
        m.delta_engine.capture("did:mesh:a", [VFSChange(path=f"/f{i}", operation="add", content_hash=f"h{i}")])
    gid = await shv.create_saga(sid)
    st = await shv.add_step(gid, "action", "did:mesh:a", "/api/action")
    await shv.execute_step(gid, st, lambda: asyncio.sleep(0))
    await shv.terminate_session(sid)


def _busy_until(kv, key: str) -> None:
    """A fixed non-hypervisor CPU load (SHA-256 over a small buffer) until ``key`` is set."""
    buf = b"x" * 4096
    n = 0
    while True:
        for _ in range(200):
            buf = hashlib.sha256(buf).digest() * 128
        n += 1
        if n % 8 == 0 and kv.check([key]):
            return


def _worker(rank: int, world: int, root: str, store: str, q) -> None:
    os.environ.update(OMP_NUM_THREADS="1", AHV_STORE=store)
    cpus = sorted(os.sched_getaffinity(0))
    if len(cpus) >= world:  # one vCPU per rank: no migrations between the timed loops
        os.sched_setaffinity(0, {cpus[rank]})
    import torch

    torch.set_num_threads(1)
    dist.init_process_group("gloo", init_method=f"file://{os.path.join(root, 'pg')}", rank=rank, world_size=world)
    from agent_hypervisor_amd.parallel.resilience import _store
    from agent_hypervisor_amd.parallel.sharded import ShardedHypervisor

    kv = _store()

    async def main():
        shv = await ShardedHypervisor(device=store).start()
        import gc

        for _ in range(50):  # warm-up
            await _pipeline(shv)
        loop = asyncio.get_running_loop()
        barrier = lambda: loop.run_in_executor(None, dist.barrier)  # noqa: E731
        gc.collect()
        gc.disable()  # no collector pauses inside the timed loops
        a_rates, a_idle, b_dts, counters = [], None, [], []

        async def phase_a(tag: str, loaded: bool):
            await barrier()
            if rank == 0:
                t0 = time.perf_counter()
                for _ in range(K):
                    await _pipeline(shv)
                rate = K / (time.perf_counter() - t0)
                kv.set(tag, "1")
                return rate
            if loaded:
                await loop.run_in_executor(None, _busy_until, kv, tag)
            return None

        for r in range(ROUNDS + 1):
            if r == 0:  # the idle-baseline round (reported, not asserted)
                a_idle = await phase_a(f"idle/{r}", loaded=False)
            else:
                a = await phase_a(f"a/{r}", loaded=True)
                if a is not None:
                    a_rates.append(a)
            await barrier()
            base = dict(shv.counters)
            t0 = time.perf_counter()
            for _ in range(K):
                await _pipeline(shv)
            b_dts.append(time.perf_counter() - t0)
            counters.append({k: shv.counters[k] - base[k] for k in base})
            gc.collect()
        gc.enable()
        kv.set(f"scale/{rank}", repr((b_dts, counters)))
        await barrier()
        if rank == 0:
            parts = [eval(kv.get(f"scale/{r}").decode()) for r in range(world)]  # noqa: S307 - own repr
            return a_rates, a_idle, parts
        return None

    res = asyncio.run(main())
    if rank == 0:
        q.put(res)
    dist.barrier()
    dist.destroy_process_group()
    q.close()
    q.join_thread()
    os._exit(0)


def _measure(tmp_path, world: int, store: str = "host"):
    os.makedirs(tmp_path, exist_ok=True)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, str(tmp_path), store, q)) for r in range(world)]
    for p in procs:
        p.start()
    a_rates, a_idle, parts = q.get(timeout=900)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    # aggregate of round r: N·K over the slowest rank's time (round 0 is the idle-baseline round)
    aggs = [world * K / max(parts[k][0][r] for k in range(world)) for r in range(ROUNDS + 1)]
    return a_rates, a_idle, aggs, [c for p in parts for c in p[1]]


@pytest.mark.slow
@pytest.mark.parametrize("world", [2, 4, 8])
def test_rank_local_serving_scales(tmp_path, world):
    """Asserted on counted work, not on a wall-clock ratio: while
    every rank serves pipelines at once, each session call is served locally —
    zero collectives, zero forwarded messages, exactly 7 local calls per pipeline
    on every rank and round.  The throughput ratio is measured and printed (it is
    the host's CPU share on a shared container, not the code's property)."""
    ncpu = len(os.sched_getaffinity(0))
    a_rates, a_idle, aggs, deltas = _measure(tmp_path / "m0", world)
    eff = statistics.median(b / (world * a) for a, b in zip(a_rates, aggs[1:]))
    print(f"world={world}: 1-rank {statistics.median(a_rates):.0f}/s (idle {a_idle:.0f}/s), aggregate "
          f"{statistics.median(aggs[1:]):.0f}/s, efficiency {eff:.2f} ({ncpu} CPUs, reported, not asserted)")
    assert len(deltas) == world * (ROUNDS + 1)
    for d in deltas:  # the per-session path never communicates
        assert d["collectives"] == 0 and d["forwarded"] == 0 and d["local"] == 7 * K, d
    assert all(r > 0 for r in a_rates) and all(b > 0 for b in aggs)


def _views_worker(rank: int, world: int, root: str, n: int, q) -> None:
    os.environ.update(OMP_NUM_THREADS="1", AHV_STORE="cpu", AHV_STORE_SESSIONS=str(1 << 18))
    import torch

    torch.set_num_threads(1)  # ranks share this host's CPUs (torch was imported before the env var)
    dist.init_process_group("gloo", init_method=f"file://{os.path.join(root, 'pg')}", rank=rank, world_size=world)
    from agent_hypervisor_amd.models.store_pipeline import PipelineSpec
    from agent_hypervisor_amd.parallel.resilience import _store
    from agent_hypervisor_amd.parallel.sharded import ShardedHypervisor
    from hypervisor import SessionConfig

    kv = _store()

    async def main():
        shv = await ShardedHypervisor(device="cpu").start()
        await shv.local.run_pipelines(PipelineSpec(), n)  # n batched sessions on this rank (archived)
        sids = [await shv.create_session(SessionConfig(), "did:admin", rank=rank) for _ in range(3)]
        for sid in sids:
            await shv.join_session(sid, "did:v0", sigma_raw=0.9)
            await shv.vouch("did:v0", f"did:x{rank}", sid, 0.9, bond_pct=0.1)
            await shv.vouch(f"did:y{rank}", "did:v0", sid, 0.8, bond_pct=0.2)
        kv.set(f"views/built/{rank}", "1")
        await asyncio.get_running_loop().run_in_executor(None, kv.wait, [f"views/built/{r}" for r in range(world)])
        if rank != 0:
            await shv.serve_forever()
            return None
        st = shv.local._store
        out = {}
        await shv.stats()  # first view: connections and the batch row caches
        for name, call in (("stats", lambda: shv.stats()), ("liability", lambda: shv.agent_liability("did:v0"))):
            p0, c0 = st.info()["posted"], dict(shv.counters)
            t0 = time.perf_counter()
            res = await call()
            dt = time.perf_counter() - t0
            out[name] = (res, st.info()["posted"] - p0, shv.counters["collectives"] - c0["collectives"], dt)
        await shv.shutdown()
        return out

    res = asyncio.run(main())
    if rank == 0:
        q.put(res)
    dist.barrier()
    dist.destroy_process_group()
    q.close()
    q.join_thread()
    os._exit(0)


def test_agent_views_cost_o1_commands_at_1e5_sessions_per_rank(tmp_path):
    """with 10⁵ sessions per rank, ``stats`` is one device
    reduction per rank plus one 48-byte all-reduce, and the owner-routed
    ``agent_liability`` reads only the agent's records (per-agent index) with no
    collective — both O(1) store commands per rank, whatever the session count."""
    world, n = 2, 100_000
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_views_worker, args=(r, world, str(tmp_path), n, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = q.get(timeout=600)
    for p in procs:
        p.join(timeout=60)
    stats, s_cmds, s_coll, s_dt = res["stats"]
    assert stats["total_sessions"] == world * (n + 3) and stats["total_sagas"] == world * n
    assert stats["active_sessions"] == world * 3 and stats["total_vouches"] == world * 6
    assert s_cmds <= 2 and s_coll == 1, (s_cmds, s_coll)
    lia, l_cmds, l_coll, l_dt = res["liability"]
    assert len(lia["vouches_given"]) == world * 3 and len(lia["vouches_received"]) == world * 3
    assert lia["total_exposure"] == sum(v["bonded_amount"] for v in lia["vouches_given"])
    assert l_cmds <= 2 and l_coll == 0, (l_cmds, l_coll)
    print(f"stats {s_dt * 1e3:.1f} ms, agent_liability {l_dt * 1e3:.1f} ms at {n} sessions per rank")
