"""Config-5 audit arena: the device-stamped per-session chains (distinct DIDs,
paths, timestamps, and a slash delta carrying the post-slash score row) hash to
exactly what the scalar DeltaEngine produces for the same session."""

from __future__ import annotations

import os
import sys
from datetime import datetime, timezone

import pytest
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
    scores_all = torch.rand((S, 16), dtype=torch.float64, generator=torch.Generator().manual_seed(1))
    scores = scores_all[touched]
    arena.write_slash_deltas(touched, scores_all)
    packed = arena.packed(touched)
    dig = A.digests_to_hex(A.chain_hashes(packed))
    # equal-length chains: the turn-major phase-1 lane order gives the same digests
    assert A.digests_to_hex(A.chain_hashes(packed, uniform_len=D + 1)) == dig
    res, sel = arena.resident(touched)
    assert A.digests_to_hex(A.chain_hashes(res, uniform_len=D + 1, sel=sel)) == dig
    with pytest.raises(ValueError):
        A.chain_hashes(res, uniform_len=D + 1, sel=torch.tensor([0, 7, 13, S]))
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


@pytest.mark.gpu
def test_arena_chains_gfx950_turn_major(cuda_device):
    """Device K08 over the arena, turn-major phase 1 (``uniform_len``) and
    consecutive lanes, against the host twin."""
    S, D = 3000, 3
    arena = AuditArena(S, D, torch.device("cuda"))
    touched = torch.arange(0, S, 7, device="cuda")
    scores = torch.rand((S, 16), dtype=torch.float64, device="cuda")
    arena.write_slash_deltas(touched, scores)
    host = AuditArena(S, D, torch.device("cpu"))
    host.write_slash_deltas(touched.cpu(), scores.cpu())
    # render_rows: device == host twin (body rows, and the rendered tail slots)
    dev_b, host_b = arena.bytes.cpu(), host.bytes
    assert torch.equal(dev_b[: S * arena.L], host_b[: S * host.L])
    slots = lambda b: b[arena.tail:].view(S, arena.pitch)[touched.cpu(), : arena.Ls]  # noqa: E731
    assert torch.equal(slots(dev_b), slots(host_b))
    packed = arena.packed(touched)
    want = A.chain_hashes(host.packed(touched.cpu()))
    assert torch.equal(A.chain_hashes(packed, uniform_len=D + 1).cpu(), want)
    res, sel = arena.resident(touched)  # spans read in place through sel
    assert torch.equal(A.chain_hashes(res, uniform_len=D + 1, sel=sel).cpu(), want)
    assert torch.equal(A.chain_hashes(res, uniform_len=D + 1, sel=sel, midstate=False).cpu(), want)
    assert torch.equal(A.chain_hashes(packed).cpu(), want)


@pytest.mark.gpu
def test_render_rows_gfx950_word_and_byte_paths(cuda_device):
    """render_rows on the device: the aligned word path (pitch multiple of 4) and
    the byte path (odd pitch) both equal the host twin."""
    g = torch.Generator().manual_seed(3)
    tmpl = torch.randint(32, 127, (101,), dtype=torch.uint8, generator=g)
    src = torch.randint(0, 256, (500, 24), dtype=torch.uint8, generator=g)
    ids = torch.randperm(500, generator=g)[:300].to(torch.int64)
    for pitch in (104, 101):
        outs = []
        for dev in ("cpu", "cuda"):
            out = torch.zeros(500 * pitch, dtype=torch.uint8, device=dev)
            A.render_rows(out, tmpl.to(dev), ids.to(dev), stamps=[(3, 7, 0, 0), (20, 6, 999_999, 1)],
                          hex_field=(40, src.to(dev), 24), pitch=pitch)
            outs.append(out.cpu())
        assert torch.equal(outs[0], outs[1]), pitch


@pytest.mark.gpu
def test_render_rows_gfx950_long_rows_and_wide_hex(cuda_device):
    """Rows longer than 64 words, several stamps, a hex field of 128 and of 300
    source bytes at an odd position: device == host twin."""
    g = torch.Generator().manual_seed(4)
    tmpl = torch.randint(32, 127, (1500,), dtype=torch.uint8, generator=g)
    src = torch.randint(0, 256, (400, 300), dtype=torch.uint8, generator=g)
    ids = torch.randperm(400, generator=g)[:257].to(torch.int64)
    for hb, pos in ((128, 401), (300, 777)):
        outs = []
        for dev in ("cpu", "cuda"):
            out = torch.zeros(400 * 1504, dtype=torch.uint8, device=dev)
            A.render_rows(out, tmpl.to(dev), ids.to(dev),
                          stamps=[(3, 7, 0, 0), (20, 6, 999_999, 1), (1490, 9, 0, 12345), (64, 18, 0, 0)],
                          hex_field=(pos, src.to(dev), hb), pitch=1504)
            outs.append(out.cpu())
        assert torch.equal(outs[0], outs[1]), hb


@pytest.mark.parametrize("dev", ["cpu", pytest.param("cuda", marks=pytest.mark.gpu)])
def test_storm_bond_update_counts_match_slashing_engine(dev):
    """Config 5's reported ``bond_updates`` are device counts: on a
    10⁴-edge instance, the full storm (every session slashed, K06 cascade, then its
    remaining bonds released, K07) changes exactly the bonds the scalar
    ``SlashingEngine.slash`` + ``VouchingEngine.release_session_bonds`` change, per
    session and in total — and that is every edge."""
    import random

    from benchmarks.bench_configs import storm_counts
    from hypervisor.liability.slashing import SlashingEngine
    from hypervisor.liability.vouching import VouchingEngine, VouchingError
    from agent_hypervisor_amd.ops import liability as LI

    T0 = datetime(2026, 3, 1, 12, tzinfo=timezone.utc)
    _clock.set_clock(lambda: T0)
    try:
        rng = random.Random(21)
        ve = VouchingEngine()
        sids, parts, sig = [], [], []
        while len(ve._vouches) < 10_000:
            s = len(sids)
            sid, p = f"s{s}", [f"did:{s}:{k}" for k in range(16)]
            sg = {d: rng.uniform(0.3, 1.0) for d in p}
            for _ in range(24):
                a, b = rng.sample(p, 2)
                try:
                    ve.vouch(a, b, sid, sg[a], bond_pct=rng.choice([0.1, 0.2, 0.3]))
                except VouchingError:
                    pass
            sids.append(sid)
            parts.append(p)
            sig.append(sg)
        E = len(ve._vouches)
        S = len(sids)
        vb = LI.from_engine(ve, sids, parts, device=dev)
        targets = [rng.randrange(16) for _ in range(S)]
        omega = torch.full((S,), 0.95, dtype=torch.float64)
        scores = torch.tensor([[sig[s][d] for d in parts[s]] for s in range(S)], dtype=torch.float64)
        now = _clock.to_us(T0)
        out = LI.slash(vb, torch.tensor(targets, dtype=torch.uint8, device=dev), omega.to(dev), scores.to(dev), now,
                       clip_cap=16, zero_records=False, with_sigma_eff=True)
        rel = LI.release_bonds(vb, now)
        counts = storm_counts(out, rel).cpu().tolist()
        se = SlashingEngine(ve)
        want_slash, want_rel = [], []
        for s, (sid, p) in enumerate(zip(sids, parts)):
            before = len(se.history)
            d = dict(sig[s])
            se.slash(p[targets[s]], sid, d[p[targets[s]]], 0.95, "storm", d)
            want_slash.append(sum(len(r.voucher_clips) for r in se.history[before:]))
            want_rel.append(ve.release_session_bonds(sid))
        assert out.clip_count.cpu().tolist() == want_slash
        assert rel.cpu().tolist() == want_rel
        assert counts == [sum(want_slash), sum(want_rel)] and sum(counts) == E >= 10_000
        assert int(vb.active.sum()) == 0 and not any(v.is_active for v in ve._vouches.values())
    finally:
        _clock.set_clock(None)
