"""Resource guards for the hot gfx950 kernels (hipFuncGetAttributes through
``_C.kernel_attributes``): the designs in csrc/ rely on these budgets, so a
compiler or source change that silently spills to scratch or grows the LDS
footprint fails here instead of showing up as a slower profile.

* governance pipeline: 3-block LDS window = (48 + 1 trash) rows × 64 lanes × 4 B,
  ≤ 168 VGPRs (3 waves/SIMD), no scratch (the saga/terminate stages run before
  the capture loop so nothing spills across the SHA rounds);
* K08 chain re-hash: same window, no scratch;
* slash (16-lane groups), σ_eff (16 threads per session), tile build: no scratch.
"""

from __future__ import annotations

import pytest

pytestmark = pytest.mark.gpu


def _attrs():
    from agent_hypervisor_amd._native import C

    return {k["name"]: k for k in C.kernel_attributes()}


def test_hot_kernels_fit_their_budgets(cuda_device):
    a = _attrs()
    pipe = a["governance_pipeline_kernel<3,3>"]
    assert pipe["lds_bytes"] == (48 + 1) * 64 * 4
    assert pipe["vgprs"] <= 168 and pipe["scratch_bytes"] == 0, pipe
    ch = a["chain_hash_kernel"]
    assert ch["lds_bytes"] == (48 + 1) * 64 * 4 and ch["scratch_bytes"] == 0, ch
    for name in ("slash_group_kernel", "sigma_eff_csr_kernel", "build_tiles_kernel", "bond_tiles_mfma_kernel",
                 "bond_fused_mfma_kernel", "merkle_tree_pass_kernel", "saga_fused_regs_kernel<10>"):
        assert a[name]["scratch_bytes"] == 0, a[name]
    assert a["slash_group_kernel"]["max_threads"] >= 256


def test_attributes_are_reported_for_every_registered_kernel(cuda_device):
    a = _attrs()
    assert len(a) >= 12
    for k in a.values():
        assert k["vgprs"] > 0 and k["max_threads"] >= 64
