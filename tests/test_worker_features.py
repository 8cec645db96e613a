"""Store-worker feature bits on gfx950 (csrc/hip/store_worker.hip): the command
wave's light result publication (bit 32), next-slot prefetch (bit 64) and the
FREE_ROWS wait narrowed to the freed rows' queued captures (bit 16) change only
*when* work happens, never *what* the device computes.

Every combination runs the same back-to-back reference pipelines
(`/root/reference/benchmarks/bench_hypervisor.py:217-239`) on a private store
with fixed, tiny tables, so session / saga / step / delta rows are reclaimed
(OP_FREE_ROWS) and reused many times while the hash engine still has captures
queued.  The oracle is the host: each capture's digest is the SHA-256 of its
canonical JSON (the device record must be those exact bytes), each root the host
Merkle root of the digests, and every row ends ARCHIVED / COMMITTED.
"""

from __future__ import annotations

import asyncio

import pytest

from agent_hypervisor_amd._native import C
from agent_hypervisor_amd.models.store import GovernanceStore
from hypervisor import Hypervisor
from hypervisor.audit.delta import SemanticDelta, delta_digest
from hypervisor.models import SessionState
from hypervisor.saga.state_machine import StepState
from tests.test_store import _pipeline

pytestmark = pytest.mark.gpu

_BITS = ("AHV_STORE_NARROW_FREE", "AHV_STORE_LIGHT_PUBLISH", "AHV_STORE_SLOT_PREFETCH")


@pytest.mark.parametrize("on", [(0, 0, 0), (1, 0, 0), (0, 1, 1), (1, 1, 1)], ids=["off", "narrow", "light+prefetch",
                                                                                  "all"])
def test_worker_feature_bits_keep_results(cuda_device, monkeypatch, on):
    for name, v in zip(_BITS, on):
        monkeypatch.setenv(name, str(v))  # read when the store's native core is built
    caps = {"S": 16, "D": 96, "E": 16, "V": 16, "G": 16, "T": 16, "B": 1 << 16}
    st = GovernanceStore("cuda", caps=caps, max_caps=dict(caps))

    async def run():
        for _ in range(150):
            hv = Hypervisor(store=st)
            s, _, ds, root, saga, step = await _pipeline(hv)
            for d in ds:
                hd = SemanticDelta(d.delta_id, d.turn_id, d.session_id, d.agent_did, d.timestamp, d.changes,
                                   d.parent_hash)
                assert d.delta_hash == delta_digest(hd)
                assert d.record() == C.delta_payload(hd)
            assert root == C.merkle_root([d.delta_hash for d in ds])
            assert s.sso.state is SessionState.ARCHIVED
            assert step.state is StepState.COMMITTED
            del s, ds, saga, step, hv  # rows go back to the store's free lists

    try:
        asyncio.run(run())
        st.drain()
        info = st.info()
        assert info["grows"] == {k: 0 for k in info["grows"]}  # every row came from reclaiming, never growth
    finally:
        st.close()
