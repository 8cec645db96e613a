"""Resource guards for the hot gfx950 kernels (hipFuncGetAttributes through
``_C.kernel_attributes``): the designs in csrc/ rely on these budgets, so a
compiler or source change that silently spills to scratch or grows the LDS
footprint fails here instead of showing up as a slower profile.

* template pipeline over store rows: 3-block LDS window = (48 + 1 trash) rows ×
  64 lanes × 4 B; the 2-waves/SIMD variant holds everything in ≤ 256 VGPRs with no
  scratch, the 3-waves variant stays within 168 VGPRs (a small spill); the small-batch
  variant holds a whole record ((96 + 1) rows) with no scratch;
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
    p2, p3 = a["store_template_kernel<2,3>"], a["store_template_kernel<3,3>"]
    assert p2["lds_bytes"] == p3["lds_bytes"] == (48 + 1) * 64 * 4
    assert p2["vgprs"] <= 256 and p2["scratch_bytes"] == 0, p2
    assert p3["vgprs"] <= 168 and p3["scratch_bytes"] <= 128, p3
    p6 = a["store_template_kernel<1,6>"]
    assert p6["lds_bytes"] == (96 + 1) * 64 * 4 and p6["scratch_bytes"] == 0, p6
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
