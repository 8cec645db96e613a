"""One device state: batched kernels over the store's resident tables.

* ``Hypervisor.verify_audit`` on a device-backed hypervisor verifies every chain
  where it lives (K10 over the arena records + d_hash rows, K09 roots from the
  resident digests): no record is re-rendered on the host and no payload byte is
  staged to the device — only int32 row lists travel.
* Batched σ_eff / exposure over the resident vouch lists equal the scalar
  commands bit for bit (reference ``liability/vouching.py:128-166``).
* The sharded X01 view reduces store edge columns on the device.
"""

from __future__ import annotations

import asyncio
import random

import pytest

from agent_hypervisor_amd.models.store import GovernanceStore
from hypervisor import Hypervisor, SessionConfig
from hypervisor.audit.delta import VFSChange


async def _sessions(hv, n: int, deltas: int = 3) -> list:
    out = []
    for i in range(n):
        m = await hv.create_session(SessionConfig(), "did:admin")
        sid = m.sso.session_id
        await hv.join_session(sid, f"did:a{i % 7}", sigma_raw=0.8)
        await hv.activate_session(sid)
        for k in range(deltas + i % 3):
            m.delta_engine.capture(f"did:a{i % 7}", [VFSChange(path=f"/f{k}", operation="add",
                                                               content_hash=f"h{i}.{k}")])
        if i % 2:
            await hv.terminate_session(sid)
        out.append(m)
    return out


def check_verify_in_place(device: str, n: int) -> None:
    from agent_hypervisor_amd.ops import audit as A

    st = GovernanceStore(device, caps={"S": 4 * n, "D": 16 * n})
    hv = Hypervisor(store=st)
    ms = asyncio.run(_sessions(hv, n))
    staged = []
    orig_stage, orig_pack = st._c.stage, A.pack_bytes
    st_stage = st.stage

    def spy_stage(data):
        staged.append(len(data))
        return st_stage(data)

    st.stage = spy_stage
    A.pack_bytes = lambda *a, **k: (_ for _ in ()).throw(AssertionError("a payload was packed on the host"))
    try:
        before = st.info()["posted"]
        rep = hv.verify_audit()
        posted = st.info()["posted"] - before
    finally:
        A.pack_bytes = orig_pack
        st.stage = st_stage
    assert rep.ok and rep.deltas == sum(m.delta_engine.turn_count for m in ms)
    assert rep.roots_checked == n // 2
    # only int32 row lists cross (the commitment view's slot list); a record is ~300 B per delta
    assert sum(staged) <= 4 * n and posted <= 8
    # tamper one resident digest: its chain (digest) and the link of its successor fail
    victim = ms[3].delta_engine.deltas[1]
    idx = [8 * victim._didx + k for k in range(8)]
    st.write_rows({"d_hash": (idx, [0x01234567] * 8)})
    rep = hv.verify_audit()
    assert rep.bad_chains == [ms[3].sso.session_id] and rep.bad_roots == [ms[3].sso.session_id]
    # the views path still re-renders (and flags edits to the Python objects)
    ms[5].delta_engine.deltas[0].agent_did = "did:forged"
    rep = hv.verify_audit(source="views")
    assert ms[5].sso.session_id in rep.bad_chains
    st.close()


def check_sigma_batch_bit_exact(device: str) -> None:
    rng = random.Random(7)
    st = GovernanceStore(device, caps={"E": 4096, "V": 64})
    hv = Hypervisor(store=st)
    v = hv.vouching
    agents = [f"did:x{i}" for i in range(12)]
    for _ in range(600):
        a, b = rng.sample(agents, 2)
        try:
            v.vouch(a, b, f"s{rng.randrange(8)}", rng.uniform(0.5, 1.0), bond_pct=rng.choice([None, rng.random()]))
        except Exception:  # noqa: BLE001 - cycles / exposure rejections are part of the workload
            pass
    for rec in rng.sample(v.records(), 40):
        v.release_bond(rec.vouch_id)
    reqs = [(rng.choice(agents), f"s{rng.randrange(9)}", rng.random(), rng.choice([0.2, 0.65, 0.95]))
            for _ in range(500)]
    got = v.compute_sigma_eff_batch(reqs)
    want = [v.compute_sigma_eff(*r) for r in reqs]
    assert got == want  # bit for bit
    ex = [(rng.choice(agents), f"s{rng.randrange(9)}") for _ in range(300)]
    assert v.get_total_exposure_batch(ex) == [v.get_total_exposure(*r) for r in ex]
    st.close()


def test_verify_in_place_cpu_twin():
    check_verify_in_place("cpu", 60)


def test_sigma_batch_bit_exact_cpu_twin():
    check_sigma_batch_bit_exact("cpu")


def test_exposure_view_over_store_edges():
    from agent_hypervisor_amd.ops.store_views import exposure_by_agent

    st = GovernanceStore("cpu", caps={"E": 256, "V": 16})
    hv = Hypervisor(store=st)
    v = hv.vouching
    v.vouch("did:a", "did:b", "s1", 0.9, bond_pct=0.3)
    v.vouch("did:a", "did:c", "s2", 0.9, bond_pct=0.2)
    r = v.vouch("did:c", "did:b", "s1", 0.8)
    v.release_bond(r.vouch_id)
    x = exposure_by_agent(st, [st.agents.lookup(d) for d in ("did:a", "did:c", "did:z")], list(v._by_edge))
    assert x.tolist() == [pytest.approx(0.9 * 0.3 + 0.9 * 0.2), 0.0, 0.0]
    st.close()


@pytest.mark.gpu
def test_verify_in_place_gpu():
    check_verify_in_place("cuda", 10_000)


@pytest.mark.gpu
def test_sigma_batch_bit_exact_gpu():
    check_sigma_batch_bit_exact("cuda")
