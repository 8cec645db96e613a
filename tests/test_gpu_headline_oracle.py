"""The production headline kernel, oracle-checked on gfx950.

``store_template_run`` takes ``store_template_kernel<1,6>`` for batches of at most
65,536 sessions and ``<3,3>`` (default), ``<2,3>`` or ``<4,2>`` above — the
variant behind the headline number.  Here each large-batch variant runs 262,144
sessions, and for 1,000 random sessions the arena records, ``d_hash``, ``s_head``
and ``s_root`` are compared with the scalar renderer + hashlib + the reference
Merkle rule (reference ``audit/delta.py:41-134``); then ``verify_audit`` re-checks
every chain and root over the arena in place (K10/K09) with no payload bytes
staged through the host.
"""

from __future__ import annotations

import numpy as np
import pytest
import torch

from agent_hypervisor_amd.models import store_template as TT

N = 262_144


@pytest.mark.parametrize("dev,waves,n", [pytest.param("cuda", 3, N, marks=pytest.mark.gpu),
                                         pytest.param("cuda", 2, N, marks=pytest.mark.gpu),
                                         pytest.param("cuda", 4, N, marks=pytest.mark.gpu),
                                         ("cpu", 3, 3000), pytest.param("cpu", 3, N, marks=pytest.mark.slow)])
def test_headline_variant_matches_the_host_oracle(dev, waves, n):
    """(The CPU case runs the host twin of the same body at a smaller batch.)"""
    from hypervisor import Hypervisor

    N = n
    hv = Hypervisor(device=dev)
    st = hv._store
    agents = TT.AgentSet.synthetic(st, 4096, seed=11, prefix=f"did:mesh:oracle{waves}-agent-")
    sa = torch.randint(0, agents.count, (N,), dtype=torch.int32, generator=torch.Generator().manual_seed(waves))
    run = TT.run(hv, N, agents=agents, session_agent=sa, variant=(waves, 0))  # small=0: never the <1,6> kernel
    assert run.ok == N
    b = hv._sessions.batch_of(run.session_ids[0])
    rng = np.random.default_rng(1000 + waves)
    pick = np.sort(rng.choice(N, size=1000, replace=False))
    tp = b.specs.tp
    assert TT.check_sessions(tp, tp.last_id_base, tp.t0, sa, pick) == 1000
    # the lazily registered sessions agree with the API's view of them
    for i in pick[:8].tolist():
        m = hv.get_session(run.session_ids[i])
        assert m.delta_engine.compute_merkle_root() == run.roots[run.session_ids[i]]
    staged = []
    orig = st.stage
    st.stage = lambda data: staged.append(len(data)) or orig(data)
    try:
        rep = hv.verify_audit()
    finally:
        st.stage = orig
    assert rep.ok and rep.deltas >= 3 * N and rep.roots_checked >= N, rep
    # row-index lists at most: no record bytes cross to the device
    assert sum(staged) <= 64 * N, sum(staged)


@pytest.mark.gpu
@pytest.mark.parametrize("n,deltas,did", [(10_000, 3, "did:mesh:coop-agent-"), (16_384, 3, "did:x:"),
                                          (5_000, 2, "did:mesh:coop2-"), (3_000, 1, "did:mesh:coop1-"),
                                          (4_000, 3, "did:mesh:a-much-longer-decentralised-identifier-")])
def test_small_batch_cooperative_kernel_matches_the_host_oracle(n, deltas, did):
    """``store_template_coop_kernel`` (batches ≤ 16,384 sessions, D ≤ 3: four waves
    per 64 sessions, records rendered at once and chained through LDS, Merkle
    level 1 beside the last record) writes the same records, digests, heads and
    roots as the scalar renderer + hashlib + the reference Merkle rule, for 6- and
    8-block records (the long DID); then verify_audit over every row."""
    from hypervisor import Hypervisor

    hv = Hypervisor(device="cuda")
    st = hv._store
    agents = TT.AgentSet.synthetic(st, 2048, seed=5, prefix=did)
    sa = torch.randint(0, agents.count, (n,), dtype=torch.int32, generator=torch.Generator().manual_seed(n))
    run = TT.run(hv, n, agents=agents, session_agent=sa, deltas=deltas)
    assert run.ok == n
    b = hv._sessions.batch_of(run.session_ids[0])
    tp = b.specs.tp
    assert tp.max_rec <= 512
    pick = np.sort(np.random.default_rng(n).choice(n, size=min(n, 1000), replace=False))
    assert TT.check_sessions(tp, tp.last_id_base, tp.t0, sa, pick) == len(pick)
    rep = hv.verify_audit()
    assert rep.ok and rep.deltas >= deltas * n, rep
