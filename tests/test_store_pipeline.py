"""Heterogeneous batched pipelines over the device store (``Hypervisor.run_pipelines``).

A randomized batch — several joins per session with per-agent σ (some refused:
capacity, σ floor, duplicates), per-delta agents and change lists, saga steps
that succeed, retry or fail, compensation with and without undo APIs, sessions
left unactivated / unterminated — must equal the scalar public API run session
by session over the same ids and timestamps, byte for byte: Merkle roots, delta
digests, session and step states, ring assignments (reference ``core.py:106-185``,
``saga/orchestrator.py:77-198``).  The batch's sessions are ordinary sessions
afterwards (views, verify, snapshots).
"""

from __future__ import annotations

import asyncio
import random

import pytest

from agent_hypervisor_amd.models.store import StoreError

from agent_hypervisor_amd.models.store import GovernanceStore
from agent_hypervisor_amd.models.store_pipeline import PipelineSpec
from hypervisor import Hypervisor, SessionConfig
from hypervisor import _clock
from hypervisor.audit.delta import VFSChange
from hypervisor.saga.orchestrator import SagaOrchestrator

AGENTS = [f"did:mesh:agent-{k}" for k in range(9)] + ["did:mesh:ünïcode\"quoted\\"]


def random_spec(rng: random.Random) -> PipelineSpec:
    joins = [(rng.choice(AGENTS), rng.choice([0.3, 0.55, 0.61, 0.7, 0.96, rng.random()]))
             for _ in range(rng.randrange(0, 6))]
    deltas = []
    for _ in range(rng.randrange(0, 5)):
        chs = [(f"/p{rng.randrange(50)}", rng.choice(["add", "update", "delete"]),
                rng.choice([None, f"h{rng.randrange(1000)}", "x" * rng.randrange(1, 90)]))
               for _ in range(rng.randrange(0, 4))]
        deltas.append((rng.choice(AGENTS), tuple(chs)))
    steps = [(f"act{k}", rng.choice(AGENTS), f"/api/{k}", rng.choice([None, f"/undo/{k}"]),
              rng.randrange(0, 3), rng.choice([0, 0, 0, 1, 2, 5])) for k in range(rng.randrange(0, 4))]
    cfg = SessionConfig(max_participants=rng.choice([2, 3, 10]), min_sigma_eff=rng.choice([0.5, 0.6, 0.9]),
                        enable_audit=rng.random() < 0.9)
    return PipelineSpec(joins=tuple(joins), deltas=tuple(deltas), steps=tuple(steps),
                        activate=rng.random() < 0.9, terminate=rng.random() < 0.85,
                        compensate=rng.random() < 0.7, config=cfg, creator_did=rng.choice(AGENTS))


async def scalar(hv, sid: str, sp: PipelineSpec, t0: int) -> dict:
    """The same pipeline through the per-call public API (clock pinned to the batch's times)."""
    out = {"rings": [], "root": None}
    _clock.set_clock(lambda: _clock.from_us(t0))
    m = await hv.create_session(sp.config or SessionConfig(), sp.creator_did, session_id=sid)
    for did, sg in sp.joins:
        try:
            out["rings"].append(int(await hv.join_session(sid, did, sigma_raw=sg)))
        except Exception:  # noqa: BLE001 - a refused join
            out["rings"].append(None)
    if sp.activate:
        try:
            await hv.activate_session(sid)
        except Exception:  # noqa: BLE001
            pass
    for k, (did, chs) in enumerate(sp.deltas):
        _clock.set_clock(lambda k=k: _clock.from_us(t0 + 1 + k))
        m.delta_engine.capture(did, [VFSChange(path=c[0], operation=c[1], content_hash=c[2]) for c in chs])
    if sp.steps:
        saga = m.saga.create_saga(sid)
        steps = [m.saga.add_step(saga.saga_id, a[0], a[1], a[2], undo_api=a[3], max_retries=a[4]) for a in sp.steps]
        failed = False
        for st_, a in zip(steps, sp.steps):
            calls = {"n": 0}

            async def ex(calls=calls, fails=a[5]):
                calls["n"] += 1
                if calls["n"] <= fails:
                    raise RuntimeError("planned failure")
                return "ok"

            try:
                await m.saga.execute_step(saga.saga_id, st_.step_id, ex)
            except RuntimeError:
                failed = True
                break
        if failed and sp.compensate:
            async def comp(step):
                return "undone"

            await m.saga.compensate(saga.saga_id, comp)
        out["steps"] = [s.state.value for s in steps]
        out["saga"] = saga.state.value
    if sp.terminate:
        try:
            out["root"] = await hv.terminate_session(sid)
        except Exception:  # noqa: BLE001
            pass
    _clock.set_clock(None)
    out["state"] = m.sso.state.value
    out["parts"] = [(p.agent_did, int(p.ring)) for p in m.sso.participants]
    out["digests"] = [d.delta_hash for d in m.delta_engine.deltas]
    return out


def batched(m) -> dict:
    out = {"state": m.sso.state.value, "parts": [(p.agent_did, int(p.ring)) for p in m.sso.participants],
           "digests": [d.delta_hash for d in m.delta_engine.deltas]}
    if m.saga.sagas:
        g = m.saga.sagas[0]
        out["steps"] = [s.state.value for s in g.steps]
        out["saga"] = g.state.value
    return out


def check_randomized(device: str, n: int, seed: int = 3) -> None:
    rng = random.Random(seed)
    specs = [random_spec(rng) for _ in range(n)]
    st = GovernanceStore(device, caps={"S": max(64, n), "D": max(256, 4 * n), "G": max(64, n), "T": max(64, 3 * n)})
    hv = Hypervisor(store=st)
    old_delay = SagaOrchestrator.DEFAULT_RETRY_DELAY_SECONDS
    SagaOrchestrator.DEFAULT_RETRY_DELAY_SECONDS = 0.0
    try:
        run = asyncio.run(hv.run_pipelines(specs))
        assert run.status.shape == (n,)
        t0 = int(hv._sessions.batch_of(run.session_ids[0]).t0)
        ref = Hypervisor(device="host")
        check = range(n) if n <= 2000 else rng.sample(range(n), 2000)
        jpos = [0]
        for sp in specs:
            jpos.append(jpos[-1] + len(sp.joins))
        for i in check:
            sid = run.session_ids[i]
            want = asyncio.run(scalar(ref, sid, specs[i], t0))
            got = batched(hv.get_session(sid))
            for k in ("state", "parts", "digests", "steps", "saga"):
                assert got.get(k) == want.get(k), (i, k, specs[i])
            codes = run.join_codes[jpos[i]:jpos[i + 1]].tolist()
            rings = run.join_rings[jpos[i]:jpos[i + 1]].tolist()
            assert [r if c == 0 else None for r, c in zip(rings, codes)] == want["rings"], (i, specs[i])
            assert run.roots.get(sid) == want["root"], (i, specs[i])
        rep = hv.verify_audit()
        assert rep.ok and rep.deltas == sum(len(s.deltas) for s in specs)
    finally:
        SagaOrchestrator.DEFAULT_RETRY_DELAY_SECONDS = old_delay
        _clock.set_clock(None)
    st.close()


def test_randomized_batch_equals_scalar_api_cpu_twin():
    check_randomized("cpu", 400)


def test_reference_template_batch_and_reuse_cpu_twin():
    st = GovernanceStore("cpu", caps={"S": 64, "D": 256, "G": 64, "T": 64},
                         max_caps={"S": 64, "D": 256, "G": 64, "T": 64})
    for _ in range(5):  # rows of dropped (never materialized) batches come back: the table never grows
        hv = Hypervisor(store=st)
        run = asyncio.run(hv.run_pipelines(PipelineSpec(), 60))
        assert run.ok == 60 and len(run.roots) == 60
        snaps = hv.snapshots()
        assert all(x.state.value == "archived" and x.participant_count == 1 for x in snaps)
        del hv, run, snaps
        import gc

        gc.collect()
    assert st.grows == {k: 0 for k in st.grows}
    st.close()


@pytest.mark.gpu
def test_randomized_batch_equals_scalar_api_gpu():
    check_randomized("cuda", 100_000)


@pytest.mark.gpu
@pytest.mark.parametrize("layout", [
    {"AHV_SP_RENDER": "coop", "AHV_SP_COOP_G": "16"},
    {"AHV_SP_RENDER": "coop", "AHV_SP_COOP_G": "4"},
    {"AHV_SP_PREFIX": "render", "AHV_SP_ORDER": "1"},
    {"AHV_SP_ORDER": "7"},
    {"AHV_SP_OVERLAP": "0"},
    {"AHV_SP_OVERLAP": "1"},
    {"AHV_SP_CHAIN_ROOTS": "0"},
    {"AHV_SP_SINK": "staged"},
    {"AHV_SP_HOIST": "0"},
    {"AHV_SP_PREFIX_PIPE": "0", "AHV_SP_CHAIN_PIPE": "0"},
])
def test_batch_kernel_layouts_render_the_same_bytes_gpu(layout):
    """The A/B layouts of the batch kernels (cooperative renderer with 16 / 4 lanes per
    record, prefix SHA inside the render pass, render lanes by record shape, rows before
    render in a pass of their own, rows beside the prefix pass, Merkle roots by the K09
    kernel, the branching arena sink, loads in line, blocks loaded then compressed) produce the same records, digests and roots as the
    scalar API (a fresh process each: the switches are read once)."""
    import os
    import subprocess
    import sys

    env = dict(os.environ, **layout)
    code = ("import sys; sys.path.insert(0, 'tests'); import test_store_pipeline as t; "
            "t.check_randomized('cuda', 20_000)")
    r = subprocess.run([sys.executable, "-c", code], cwd=os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                       env=env, capture_output=True, text=True, timeout=280)
    assert r.returncode == 0, r.stderr[-3000:]


def check_status_precedence(device: str, render_first: int) -> None:
    import numpy as np

    from agent_hypervisor_amd.models import store_pipeline as SP

    st = GovernanceStore(device, caps={"S": 64, "D": 256, "G": 64, "T": 64})
    hv = Hypervisor(store=st)
    dup = (("did:mesh:a", 0.9), ("did:mesh:a", 0.9))  # the second join is a duplicate: join_refused
    specs = [PipelineSpec(), PipelineSpec(), PipelineSpec(joins=dup), PipelineSpec(), PipelineSpec(joins=dup)]
    p = SP.prepare(hv, specs)
    p.args["render_first"] = render_first
    p.args["chain_roots"] = int(render_first != 0)
    s_state = st.tables["s_state"]
    s_state[int(p.slots[1])] = 1  # held by someone else
    dcap = p.tens["dcap"]
    d_off = list(p.delta_off)
    for i in (2, 3):  # the session's last record gets one 64-byte line: it overflows
        dcap[d_off[i + 1] - 1] = 64
    SP.launch(p)
    status = p.tens["status"].cpu().numpy()
    assert status.tolist() == [0, 1, 6, 6, 2]
    assert int(s_state[int(p.slots[1])]) == 1  # not written
    mb = p.tens["mid_blocks"].cpu().numpy()
    assert not mb[d_off[1]:d_off[2]].any()  # the refused row's records were not hashed
    assert mb[d_off[0]:d_off[1]].all() and np.asarray(mb[d_off[4]:d_off[5]]).all()
    del hv, p
    st.close()


@pytest.mark.parametrize("render_first", [0, 1, 2])
def test_status_codes_and_precedence_in_every_kernel_order(render_first):
    """Rows pass first (0), the rows blocks beside the prefix SHA pass (1) or beside the
    render pass (2, default: codes meet through atomicMax): a row the store holds is
    refused whole (row_in_use), a record past its reservation reports record_overflow —
    over a refused join too — and the other sessions of the batch run through (CPU twin
    of the device order)."""
    check_status_precedence("cpu", render_first)


@pytest.mark.gpu
@pytest.mark.parametrize("render_first", [0, 1, 2])
def test_status_codes_and_precedence_in_every_kernel_order_gpu(render_first):
    check_status_precedence("cuda", render_first)


def test_lazy_rows_released_in_bulk_and_materialized_rows_kept(monkeypatch):
    import gc

    from agent_hypervisor_amd.models import store_pipeline as SP

    monkeypatch.setattr(SP._Batch, "_FLUSH", 7)
    st = GovernanceStore("cpu", caps={"S": 128, "D": 512, "G": 128, "T": 128})
    base = {k: st.live_rows()[k] for k in ("S", "G", "T", "D")}
    hv = Hypervisor(store=st)
    run = asyncio.run(hv.run_pipelines(PipelineSpec(), 40))
    keep = [hv.get_session(sid) for sid in run.session_ids[:5]]
    assert all(len(m.delta_engine.deltas) == 3 for m in keep)  # materialized: they own their rows
    for sid in run.session_ids[5:25]:  # dropped one by one: released every _FLUSH
        hv._sessions.pop(sid)
    gc.collect()
    st.reclaim()
    assert st.live_rows()["S"] == base["S"] + 40 - 14  # two flushes of 7; 6 wait for the batch
    del hv, run  # row lifetime follows the hypervisor: the held views' rows go with it
    gc.collect()
    st.reclaim()
    assert {k: st.live_rows()[k] for k in ("S", "G", "T", "D")} == base
    assert [m.sso.session_id for m in keep] and all(m.delta_engine.deltas[2].delta_id == "delta:3" for m in keep)
    with pytest.raises(StoreError, match="closed Hypervisor"):
        keep[0].sso.participants
    del keep
    gc.collect()
    st.reclaim()
    assert {k: st.live_rows()[k] for k in ("S", "G", "T", "D")} == base
    st.close()


def test_batch_sessions_verify_and_search_without_building_views():
    st = GovernanceStore("cpu", caps={"S": 256, "D": 1024, "G": 256, "T": 256})
    hv = Hypervisor(store=st)
    run = asyncio.run(hv.run_pipelines(PipelineSpec(), 100))
    b = hv._sessions.batch_of(run.session_ids[0])
    rep = hv.verify_audit()
    assert rep.ok and rep.deltas == 300 and rep.roots_checked == 100
    assert hv.find_saga("saga:none") == (None, None)
    assert not b.views  # nothing was materialized
    m = hv.get_session(run.session_ids[7])
    sg = m.saga.sagas[0]
    assert hv.find_saga(sg.saga_id)[1] is sg and len(b.views) == 1
    st.write_rows({"d_hash": ([8 * int(b.drows[3 * 9 + 1])], [0x0BADBEEF])})  # corrupt session 9's 2nd digest
    rep = hv.verify_audit()
    assert rep.bad_chains == [run.session_ids[9]] and rep.bad_roots == [run.session_ids[9]]
    st.close()


def test_batch_saga_summaries_without_views_match_built_views():
    st = GovernanceStore("cpu", caps={"S": 256, "D": 1024, "G": 256, "T": 256})
    hv = Hypervisor(store=st)
    rng = random.Random(3)
    specs = [random_spec(rng) for _ in range(60)]
    run = asyncio.run(hv.run_pipelines(specs))
    lazy = hv.saga_summaries()
    b = hv._sessions.batch_of(run.session_ids[0])
    assert not b.views
    built = hv.saga_summaries([hv.get_session(sid) for sid in run.session_ids if hv.get_session(sid) is not None])
    assert len(b.views) == 60
    key = lambda d: d["session_id"]  # noqa: E731
    assert sorted(lazy, key=key) == sorted(built, key=key)
    st.close()


def test_dashboard_and_stats_over_batches_build_no_views():
    from fastapi.testclient import TestClient

    from hypervisor.api.server import create_app

    st = GovernanceStore("cpu", caps={"S": 1024, "D": 4096, "G": 1024, "T": 1024})
    hv = Hypervisor(store=st)
    run = asyncio.run(hv.run_pipelines(PipelineSpec(), 500))
    b = hv._sessions.batch_of(run.session_ids[0])
    app = create_app(hv)
    with TestClient(app) as c:
        s = c.get("/api/v1/stats").json()
        assert s["total_sessions"] == 500
        d = c.get("/api/v1/dashboard/summary").json()
    assert not b.views
    assert d["overview"]["sessions"] == 500
    st.close()


@pytest.mark.parametrize("threads", [2, 4, 8])
def test_parallel_spec_walk_packs_the_serial_columns(threads):
    """pack_specs' GIL-free parallel walk (disjoint spec ranges per thread, strings
    merged in first-occurrence order) yields the serial walk's columns and pool ids,
    with non-ASCII strings (encoded by the merge) and a spec off the fast shapes
    (a list config field read through the attribute protocol → serial redo)."""
    from agent_hypervisor_amd._native import C
    from agent_hypervisor_amd.models import store_pipeline as SP

    rng = random.Random(11)
    specs = [random_spec(rng) for _ in range(3000)]
    specs[5] = PipelineSpec(joins=(("did:mesh:été", 0.7),), deltas=(("did:mesh:été", (("/ü", "add", None),)),),
                            steps=(), config=None)

    def pack(sp, th):
        a, p = C.StringPool(), C.StringPool()
        out = C.pack_specs(sp, a, p, lambda c: (4, 0.5, 1), SP._FIXED, th)
        return out, [a.str(i) for i in range(len(a))], [p.str(i) for i in range(len(p))]

    ref = pack(specs, 1)
    got = pack(specs, threads)
    assert got[1] == ref[1] and got[2] == ref[2]
    assert all(got[0][k] == ref[0][k] for k in ref[0])

    class Odd:  # a spec object without an instance __dict__ entry for its fields
        joins, deltas, steps, activate, terminate, compensate, config, creator_did = (
            (), (), (), True, True, True, None, "did:mesh:odd")

    mixed = specs[:100] + [Odd()] + specs[100:200]
    assert all(pack(mixed, threads)[0][k] == pack(mixed, 1)[0][k] for k in ref[0])


def test_spec_walk_is_version_guarded():
    """the GIL-free walk reads instance dicts through
    ``_PyObject_GetDictPtr``, which materialises (allocates) a dict on Python ≥ 3.11;
    the extension compiles it in only below 3.11 and takes the serial walk otherwise,
    and the forced serial walk gives the parallel walk's columns and pool ids."""
    import sys

    from agent_hypervisor_amd._native import C
    from agent_hypervisor_amd.models import store_pipeline as SP

    rng = random.Random(3)
    specs = [random_spec(rng) for _ in range(2000)]

    def pack(th):
        a, p = C.StringPool(), C.StringPool()
        out = C.pack_specs(specs, a, p, lambda c: (4, 0.5, 1), SP._FIXED, th)
        return out, [a.str(i) for i in range(len(a))], [p.str(i) for i in range(len(p))], C.pack_walk_info()[1]

    compiled, _ = C.pack_walk_info()
    assert compiled == (sys.version_info < (3, 11))
    ser, par = pack(1), pack(4)
    assert ser[3] == "serial" and par[3] == ("parallel" if compiled else "serial")
    assert ser[1] == par[1] and ser[2] == par[2] and all(ser[0][k] == par[0][k] for k in ser[0])
