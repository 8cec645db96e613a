"""Config-5 audit arena: the device-stamped per-session chains (distinct DIDs,
paths, timestamps, and a slash delta carrying the post-slash score row) hash to
exactly what the scalar DeltaEngine produces for the same session."""

from __future__ import annotations

import os
import sys
from datetime import datetime, timezone

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from agent_hypervisor_amd.ops import audit as A  # noqa: E402
from benchmarks.bench_configs import AuditArena  # noqa: E402
from hypervisor import _clock  # noqa: E402
from hypervisor.audit.delta import DeltaEngine, VFSChange  # noqa: E402


def test_arena_chains_match_scalar_delta_engine():
    S, D = 40, 3
    arena = AuditArena(S, D, torch.device("cpu"))
    touched = torch.tensor([0, 7, 13, 39])
    scores = torch.rand((4, 16), dtype=torch.float64, generator=torch.Generator().manual_seed(1))
    arena.write_slash_deltas(touched, scores)
    packed = arena.packed(touched)
    dig = A.digests_to_hex(A.chain_hashes(packed))
    for i, s in enumerate(touched.tolist()):
        tag = f"{s:07d}"
        _clock.set_clock(lambda s=s: datetime(2026, 3, 1, 12, 0, 0, s % 999_999 + 1, tzinfo=timezone.utc))
        de = DeltaEngine(f"session:{tag}")
        for k in range(D):
            de.capture(f"did:mesh:agent-{tag}", [VFSChange(f"/s{tag}/f{k}", "add", f"h{k}-{tag}")])
        hexrow = scores[i].contiguous().view(torch.uint8).numpy().tobytes().hex()
        de.capture(f"did:mesh:agent-{tag}", [VFSChange(f"/s{tag}/slash", "modify", hexrow)])
        assert dig[i * (D + 1):(i + 1) * (D + 1)] == [d.delta_hash for d in de.deltas], s
        roots = A.merkle_roots(packed["chain_offsets"], A.chain_hashes(packed))
        assert A.digests_to_hex(roots[i:i + 1])[0] == de.compute_merkle_root()
    _clock.set_clock(None)
