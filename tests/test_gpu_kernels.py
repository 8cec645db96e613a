"""gfx950 kernels K01–K22 == their host twins (same element bodies, run on the
CPU in tests/test_kernels_host.py against the Python engines)."""

from __future__ import annotations

import random

import pytest
import torch

from agent_hypervisor_amd.ops import audit as A
from agent_hypervisor_amd.ops import ledger as L
from agent_hypervisor_amd.ops import liability as LI
from agent_hypervisor_amd.ops import rings as R
from agent_hypervisor_amd.ops import saga as SG
from agent_hypervisor_amd.ops import security as SEC
from agent_hypervisor_amd.ops import session as SE

pytestmark = pytest.mark.gpu
f64, u8, i32, i64 = torch.float64, torch.uint8, torch.int32, torch.int64


def _both(fn, *tensors):
    """Run ``fn`` on CPU copies and on cuda copies of ``tensors``; returns both
    (outputs, mutated inputs) on the CPU."""
    cpu = [t.clone() for t in tensors]
    dev = [t.clone().cuda() for t in tensors]
    out_c = fn(*cpu)
    out_d = fn(*dev)
    torch.cuda.synchronize()
    return (out_c, cpu), (_to_cpu(out_d), [t.cpu() for t in dev])


def _to_cpu(x):
    if isinstance(x, torch.Tensor):
        return x.cpu()
    if isinstance(x, (tuple, list)):
        return type(x)(_to_cpu(v) for v in x)
    if isinstance(x, dict):
        return {k: _to_cpu(v) for k, v in x.items()}
    if hasattr(x, "__dataclass_fields__"):
        return {k: _to_cpu(getattr(x, k)) for k in x.__dataclass_fields__}
    return x


def _eq(a, b, exact=True):
    a, b = _to_cpu(a), _to_cpu(b)
    if isinstance(a, torch.Tensor):
        if exact:
            assert torch.equal(a, b) or (a.is_floating_point() and torch.equal(a.nan_to_num(7.0), b.nan_to_num(7.0)))
        else:
            torch.testing.assert_close(a, b, rtol=0, atol=1e-12, equal_nan=True)
    elif isinstance(a, (tuple, list)):
        for x, y in zip(a, b):
            _eq(x, y, exact)
    elif isinstance(a, dict):
        for k in a:
            _eq(a[k], b[k], exact)
    else:
        assert a == b


def _check(fn, *tensors, exact=True):
    (oc, ic), (od, idv) = _both(fn, *tensors)
    _eq(oc, od, exact)
    _eq(ic, idv, exact)


def test_ring_kernels(cuda_device):
    g = torch.Generator().manual_seed(0)
    n = 100_000
    sig = torch.rand(n, dtype=f64, generator=g)
    cons = torch.randint(0, 2, (n,), dtype=u8, generator=g)
    _check(lambda s, c: R.ring_gate(s, c), sig, cons)
    ring = torch.randint(0, 4, (n,), dtype=u8, generator=g)
    flags = torch.randint(0, 8, (n,), dtype=u8, generator=g)
    wit = torch.randint(0, 2, (n,), dtype=u8, generator=g)
    _check(lambda *t: R.ring_check(*t), ring, flags, sig, cons, wit)


def _vouch_batch(S, seed, lo=0, hi=40):
    rng = random.Random(seed)
    offs, vr, ve, bd, ac, ex = [0], [], [], [], [], []
    for _ in range(S):
        for _ in range(rng.randint(lo, hi)):
            a, b = rng.sample(range(16), 2)
            vr.append(a)
            ve.append(b)
            bd.append(rng.uniform(0.0, 0.4))
            ac.append(int(rng.random() < 0.9))
            ex.append(rng.choice([-1, -1, 50, 150]))
        offs.append(len(vr))
    return LI.VouchBatch(torch.tensor(offs, dtype=i32), torch.tensor(vr, dtype=u8), torch.tensor(ve, dtype=u8),
                         torch.tensor(bd, dtype=f64), torch.tensor(ac, dtype=u8), torch.tensor(ex, dtype=i64),
                         torch.zeros(len(vr), dtype=i64))


def test_liability_kernels(cuda_device):
    S = 2048
    vb = _vouch_batch(S, 1)
    g = torch.Generator().manual_seed(1)
    sigma = torch.rand((S, 16), dtype=f64, generator=g)
    omega = torch.rand(S, dtype=f64, generator=g)
    fields = list(vb.__dataclass_fields__)

    def mk(*t):
        return LI.VouchBatch(*t[: len(fields)])

    _check(lambda *t: LI.build_tiles(mk(*t), 100), *[getattr(vb, f) for f in fields])
    _check(lambda *t: LI.sigma_eff_exact(mk(*t[:-2]), t[-2], t[-1], 100), *[getattr(vb, f) for f in fields],
           sigma, omega)
    tiles = LI.build_tiles(vb, 100)
    # MFMA sums in tile order; host twin sums sequentially — same terms, fp64
    _check(lambda t, s, o: LI.bond_tiles(t, s, o), tiles, sigma, omega, exact=False)
    ref = LI.sigma_eff_exact(vb, sigma, omega, 100)
    se, _, _ = LI.bond_tiles(tiles.cuda(), sigma.cuda(), omega.cuda())
    torch.testing.assert_close(se.cpu(), ref, rtol=0, atol=1e-12)
    # fused agent-indexed exposure scatter (X01 input) == index_add of the per-session rows
    members = torch.randint(0, 500, (S, 16), generator=g)
    agent_x = torch.zeros(500, dtype=f64, device="cuda")
    _, expo, _ = LI.bond_tiles(tiles.cuda(), sigma.cuda(), omega.cuda(), members=members.cuda(), agent_exposure=agent_x)
    want = torch.zeros(500, dtype=f64).index_add_(0, members.reshape(-1), expo.cpu().reshape(-1))
    torch.testing.assert_close(agent_x.cpu(), want, rtol=1e-12, atol=1e-12)
    host_x = torch.zeros(500, dtype=f64)
    LI.bond_tiles(tiles, sigma, omega, members=members, agent_exposure=host_x)
    torch.testing.assert_close(host_x, want, rtol=1e-12, atol=1e-12)
    _check(lambda *t: LI.release_bonds(mk(*t), 100), *[getattr(vb, f) for f in fields])
    tgt = torch.randint(0, 16, (S,), dtype=u8, generator=g)
    scores = torch.rand((S, 16), dtype=f64, generator=g)
    scores[scores < 0.1] = float("nan")
    _check(lambda *t: LI.slash(mk(*t[:-3]), t[-3], t[-2], t[-1], 100), *[getattr(vb, f) for f in fields],
           tgt, omega, scores)
    # admission
    rng = random.Random(2)
    r_off, rv, re_, rs, rp = [0], [], [], [], []
    for _ in range(S):
        for _ in range(rng.randint(0, 12)):
            rv.append(rng.randrange(16))
            re_.append(rng.randrange(16))
            rs.append(rng.uniform(0.3, 1.0))
            rp.append(rng.choice([0.1, 0.2, 0.5]))
        r_off.append(len(rv))
    _check(lambda *t: LI.vouch_admit(mk(*t[: len(fields)]), *t[len(fields):], 100),
           *[getattr(vb, f) for f in fields], torch.tensor(r_off, dtype=i32), torch.tensor(rv, dtype=u8),
           torch.tensor(re_, dtype=u8), torch.tensor(rs, dtype=f64), torch.tensor(rp, dtype=f64))


@pytest.mark.parametrize("S,lo,hi", [(2047, 0, 40), (96, 0, 700), (5, 0, 3)])
def test_bond_fused_mfma(cuda_device, S, lo, hi):
    """K03/K04 fused CSR → MFMA vs the creation-order CSR path (σ_eff, 1e-12) and
    the host twin (exposure / bonded_in / agent scatter); ragged tails (S not a
    multiple of the 16-session wave group), empty and > 512-edge sessions."""
    vb = _vouch_batch(S, 11 + S, lo=lo, hi=hi)
    g = torch.Generator().manual_seed(S)
    sigma = torch.rand((S, 16), dtype=f64, generator=g)
    sigma[sigma < 0.05] = float("nan")  # absent agents read as 0
    omega = torch.rand(S, dtype=f64, generator=g)
    members = torch.randint(0, 300, (S, 16), generator=g)
    ref = LI.sigma_eff_exact(vb, sigma, omega, 100)
    hx = torch.zeros(300, dtype=f64)
    h_se, h_ex, h_bi = LI.bond_fused(vb, sigma, omega, 100, members=members, agent_exposure=hx, bonded_in=True)
    assert torch.equal(h_se, ref)
    dx = torch.zeros(300, dtype=f64, device="cuda")
    d_se, d_ex, d_bi = LI.bond_fused(vb.to("cuda"), sigma.cuda(), omega.cuda(), 100, members=members.cuda(),
                                     agent_exposure=dx, bonded_in=True)
    torch.testing.assert_close(d_se.cpu(), ref, rtol=0, atol=1e-12)
    torch.testing.assert_close(d_ex.cpu(), h_ex, rtol=0, atol=1e-12)
    torch.testing.assert_close(d_bi.cpu(), h_bi, rtol=0, atol=1e-12)
    torch.testing.assert_close(dx.cpu(), hx, rtol=1e-12, atol=1e-12)
    tiles = LI.build_tiles(vb, 100)  # the old two-kernel pair gives the same exposure
    _, t_ex, _ = LI.bond_tiles(tiles, sigma.nan_to_num(0.0), omega)
    torch.testing.assert_close(h_ex, t_ex, rtol=0, atol=1e-12)


def test_liability_kernels_large_sessions(cuda_device):
    """Sessions past every staging limit: > 64 edges (slash falls back from the
    16-lane group form to one lane), > 512 (tile build reads global memory),
    > 2048 per 16-session block (σ_eff element form), mixed with small ones in
    the same blocks; duplicate (voucher, vouchee) pairs compound."""
    S = 96
    vb = _vouch_batch(S, 7, lo=0, hi=700)
    fields = list(vb.__dataclass_fields__)
    g = torch.Generator().manual_seed(7)
    sigma = torch.rand((S, 16), dtype=f64, generator=g)
    omega = torch.rand(S, dtype=f64, generator=g)

    def mk(*t):
        return LI.VouchBatch(*t[: len(fields)])

    assert int((vb.offsets[1:] - vb.offsets[:-1]).max()) > 512
    _check(lambda *t: LI.build_tiles(mk(*t), 100), *[getattr(vb, f) for f in fields])
    _check(lambda *t: LI.sigma_eff_exact(mk(*t[:-2]), t[-2], t[-1], 100), *[getattr(vb, f) for f in fields],
           sigma, omega)
    tgt = torch.randint(0, 16, (S,), dtype=u8, generator=g)
    scores = torch.rand((S, 16), dtype=f64, generator=g)
    scores[scores < 0.1] = float("nan")
    _check(lambda *t: LI.slash(mk(*t[:-3]), t[-3], t[-2], t[-1], 100), *[getattr(vb, f) for f in fields],
           tgt, omega, scores)
    # storm subsets: target 255 leaves a session untouched
    tgt2 = tgt.clone()
    tgt2[::3] = 255
    _check(lambda *t: LI.slash(mk(*t[:-3]), t[-3], t[-2], t[-1], 100), *[getattr(vb, f) for f in fields],
           tgt2, omega, scores)
    # fused K06+K03 (σ_eff in the slash pass): device == host twin == unfused, bit for bit,
    # across the 16-lane group form, the > 64-edge fallback and untouched sessions
    vd = vb.to("cuda")
    fd = LI.slash(vd, tgt2.cuda(), omega.cuda(), scores.cuda(), 100, with_sigma_eff=True)
    vh = LI.VouchBatch(*[getattr(vb, f).clone() for f in fields])
    fh = LI.slash(vh, tgt2, omega, scores.clone(), 100, with_sigma_eff=True)
    vs = LI.VouchBatch(*[getattr(vb, f).clone() for f in fields])
    sh = LI.slash(vs, tgt2, omega, scores.clone(), 100)
    assert torch.equal(fh.sigma_eff, LI.sigma_eff_exact(vs, sh.scores, omega, 100))
    assert torch.equal(fd.sigma_eff.cpu(), fh.sigma_eff)
    torch.testing.assert_close(fd.scores.cpu(), fh.scores, rtol=0, atol=0, equal_nan=True)  # NaN = absent
    assert torch.equal(vd.active.cpu(), vh.active)
    # admission past the 1024-edge LDS stage (global-memory fallback) mixed with staged blocks
    rng = random.Random(9)
    r_off, rv, re_, rs, rp = [0], [], [], [], []
    for _ in range(S):
        for _ in range(rng.randint(0, 20)):
            rv.append(rng.randrange(16))
            re_.append(rng.randrange(16))
            rs.append(rng.uniform(0.3, 1.0))
            rp.append(rng.choice([0.05, 0.1, 0.5]))
        r_off.append(len(rv))
    _check(lambda *t: LI.vouch_admit(mk(*t[: len(fields)]), *t[len(fields):], 100),
           *[getattr(vb, f) for f in fields], torch.tensor(r_off, dtype=i32), torch.tensor(rv, dtype=u8),
           torch.tensor(re_, dtype=u8), torch.tensor(rs, dtype=f64), torch.tensor(rp, dtype=f64))


def test_audit_kernels(cuda_device):
    import hashlib

    rng = random.Random(3)
    msgs = [bytes(rng.randrange(256) for _ in range(rng.choice([0, 1, 55, 56, 64, 119, 200, 1500])))
            for _ in range(3000)]
    data, offs = A.pack_bytes(msgs)
    dig = A.sha256_many(data.cuda(), offs.cuda())
    assert A.digests_to_hex(dig) == [hashlib.sha256(m).hexdigest() for m in msgs]
    # merkle over ragged chains
    leaves = torch.randint(-(2**31), 2**31 - 1, (5000, 8), dtype=i32)
    cuts = sorted(rng.sample(range(1, 5000), 700))
    moffs = torch.tensor([0] + cuts + [5000], dtype=i32)
    _check(lambda o, l: A.merkle_roots(o, l), moffs, leaves)
    # verify: chains of random payloads with correct links, some tampered
    pays = [bytes(rng.randrange(256) for _ in range(rng.randint(100, 400))) for _ in range(4000)]
    hexes = [hashlib.sha256(p).hexdigest() for p in pays]
    chain_offs = [0] + sorted(rng.sample(range(1, 4000), 500)) + [4000]
    parent, has_parent = [], []
    for c in range(len(chain_offs) - 1):
        for i in range(chain_offs[c], chain_offs[c + 1]):
            has_parent.append(int(i != chain_offs[c]))
            parent.append(hexes[i - 1] if i != chain_offs[c] else "0" * 64)
    for k in rng.sample(range(4000), 40):
        hexes[k] = "ab" * 32
    # K08 chain re-derivation: device == host on real delta chains
    from hypervisor.audit.delta import DeltaEngine, VFSChange

    chains = []
    for s in range(300):
        de = DeltaEngine(f"session:{s}")
        for t in range(rng.randint(1, 12)):
            de.capture(f"did:a{t}", [VFSChange(f"/p{t}", "modify", f"h{t}", f"g{t}")])
        chains.append(de.deltas)
    packed = A.pack_chains(chains)
    hc = A.chain_hashes(packed)
    hd = A.chain_hashes({k: v.cuda() for k, v in packed.items()})
    assert torch.equal(hc, hd.cpu())
    hs = A.chain_hashes({k: v.cuda() for k, v in packed.items()}, midstate=False)
    assert torch.equal(hc, hs.cpu())
    # midstate split with prefixes of 2-8 whole blocks (more than one 4-block LDS
    # staging round) at every byte alignment of the arena
    long_chains = []
    for s in range(700):
        de = DeltaEngine(f"session:{s}")
        for t in range(rng.randint(1, 6)):
            de.capture("did:" + "x" * rng.randint(1, 330), [VFSChange(f"/p{t}", "add", "h" * rng.randint(0, 90))])
        long_chains.append(de.deltas)
    lp = A.pack_chains(long_chains)
    assert {int(x) % 4 for x in lp["pre_off"]} == {0, 1, 2, 3} and int(lp["pre_len"].max()) >= 7 * 64
    ld = A.chain_hashes({k: v.cuda() for k, v in lp.items()})
    assert A.digests_to_hex(ld.cpu()) == [d.delta_hash for c in long_chains for d in c]
    assert A.digests_to_hex(hc) == [d.delta_hash for c in chains for d in c]
    d, o = A.pack_bytes(pays)
    _check(lambda *t: A.verify_chains(*t), d, o, A.hex_to_digests(hexes), A.hex_to_digests(parent),
           torch.tensor(has_parent, dtype=u8), torch.tensor(chain_offs, dtype=i32))


def test_saga_kernels(cuda_device):
    g = torch.Generator().manual_seed(4)
    n = 50_000
    st = torch.randint(0, 7, (n,), dtype=u8, generator=g)
    tg = torch.randint(0, 7, (n,), dtype=u8, generator=g)
    _check(lambda s, t, a, b: SG.transition(s, t, 9, started_us=a, completed_us=b), st, tg,
           torch.zeros(n, dtype=i64), torch.zeros(n, dtype=i64))
    st5 = torch.randint(0, 5, (n,), dtype=u8, generator=g)
    tg5 = torch.randint(0, 5, (n,), dtype=u8, generator=g)
    _check(lambda s, t, b: SG.transition(s, t, 9, saga=True, completed_us=b), st5, tg5, torch.zeros(n, dtype=i64))
    G = 10_000
    sizes = torch.randint(0, 9, (G,), generator=g)
    offs = torch.cat([torch.zeros(1, dtype=torch.int64), sizes.cumsum(0)]).to(i32)
    _check(lambda o, p, s: SG.fanout_policy(o, p, s), offs, torch.randint(0, 3, (G,), dtype=u8, generator=g),
           torch.randint(0, 2, (int(offs[-1]),), dtype=u8, generator=g))


def test_security_kernels(cuda_device):
    g = torch.Generator().manual_seed(5)
    n, cap = 4096, 64
    prof = SEC.BreachProfiles.allocate(n, cap, ring_counts=True)
    fields = list(prof.__dataclass_fields__)
    t = torch.zeros(n, dtype=i64)
    cpu_p = SEC.BreachProfiles(*[getattr(prof, f).clone() for f in fields])
    dev_p = SEC.BreachProfiles(*[getattr(prof, f).clone().cuda() for f in fields])
    for step in range(80):
        t = t + torch.randint(100_000, 20_000_000, (n,), generator=g)
        ar = torch.randint(1, 4, (n,), dtype=u8, generator=g)
        cr = torch.randint(0, 4, (n,), dtype=u8, generator=g)
        oc = SEC.breach_record(cpu_p, t, ar, cr)
        od = SEC.breach_record(dev_p, t.cuda(), ar.cuda(), cr.cuda())
        _eq(oc, od)
    _eq(cpu_p, dev_p)
    m = 100_000
    _check(lambda *a: SEC.token_bucket(*a, 1_000_000), torch.rand(m, dtype=f64, generator=g) * 10,
           torch.zeros(m, dtype=i64), torch.full((m,), 10.0, dtype=f64), torch.rand(m, dtype=f64, generator=g),
           torch.rand(m, dtype=f64, generator=g) * 3)
    _check(lambda a, e, r: SEC.expiry_tick(a, e, 500, r), torch.randint(0, 2, (m,), dtype=u8, generator=g),
           torch.randint(-1, 1000, (m,), dtype=i64, generator=g), torch.zeros(m, dtype=i64))


def test_ledger_kernels(cuda_device):
    g = torch.Generator().manual_seed(6)
    A_ = 20_000
    sizes = torch.randint(0, 12, (A_,), generator=g)
    offs = torch.cat([torch.zeros(1, dtype=torch.int64), sizes.cumsum(0)]).to(i32)
    E = int(offs[-1])
    _check(lambda o, t, s: L.risk_profiles(o, t, s), offs, torch.randint(0, 9, (E,), dtype=u8, generator=g),
           torch.rand(E, dtype=f64, generator=g))
    _check(lambda d: L.drift_severity(d), torch.rand(100_000, dtype=f64, generator=g))
    C = 5000
    nn = torch.randint(1, 12, (C,), generator=g)
    na = torch.randint(1, 6, (C,), generator=g)
    noffs = torch.cat([torch.zeros(1, dtype=torch.int64), nn.cumsum(0)]).to(i32)
    aoffs = torch.cat([torch.zeros(1, dtype=torch.int64), na.cumsum(0)]).to(i32)
    aon = torch.cat([torch.randint(0, int(na[c]), (int(nn[c]),), generator=g) for c in range(C)]).to(i32)
    N = int(noffs[-1])
    _check(lambda *t: L.attribution_raw(*t), noffs, aoffs, aon, torch.randint(0, 2, (N,), dtype=u8, generator=g),
           torch.randint(0, 2, (N,), dtype=u8, generator=g), torch.rand(N, dtype=f64, generator=g))


def test_session_kernels(cuda_device):
    g = torch.Generator().manual_seed(7)
    G, P, Ag, per = 512, 6, 40, 50
    offs = torch.arange(0, (G + 1) * per, per, dtype=i32)
    n = G * per
    grp = torch.arange(n) // per
    op = torch.randint(0, 2, (n,), dtype=u8, generator=g)
    col = torch.randint(0, Ag, (n,), generator=g)
    path = (grp * P + torch.randint(0, P, (n,), generator=g)).to(i32)
    agent = (grp * Ag + col).to(i32)
    _check(lambda *t: SE.vector_clock_ops(*t), offs, op, path, agent, col.to(i32),
           torch.zeros((G * P, Ag), dtype=i32), torch.zeros((G * Ag, Ag), dtype=i32))
    R_, Lk = 1000, 8000
    rs = torch.randint(0, 16, (R_,), generator=g)
    roffs = torch.cat([torch.zeros(1, dtype=torch.int64), rs.cumsum(0)]).to(i32)
    Lk = int(roffs[-1])
    m = 50_000
    _check(lambda *t: SE.lock_conflicts(*t), roffs, torch.randint(0, 30, (Lk,), dtype=i32, generator=g),
           torch.randint(0, 3, (Lk,), dtype=u8, generator=g), torch.randint(0, R_, (m,), dtype=i32, generator=g),
           torch.randint(0, 30, (m,), dtype=i32, generator=g), torch.randint(0, 3, (m,), dtype=u8, generator=g))


def test_spread_fold(cuda_device):
    """Single-wave spread-counter fold: sum of the 64 rows added / copied, rows re-zeroed."""
    from agent_hypervisor_amd.utils.stats import SpreadCounters

    sc = SpreadCounters(6, cuda_device)
    rows = torch.randint(0, 1 << 40, (64, 6), dtype=torch.int64)
    sc.buf.copy_(rows)
    out = torch.arange(6, dtype=torch.int64, device=cuda_device)
    sc.add_into(out)
    torch.cuda.synchronize()
    assert out.cpu().tolist() == (rows.sum(0) + torch.arange(6)).tolist()
    assert int(sc.buf.abs().sum()) == 0
    sc.buf.copy_(rows)
    sc.copy_into(out)
    torch.cuda.synchronize()
    assert out.cpu().tolist() == rows.sum(0).tolist()
    assert int(sc.buf.abs().sum()) == 0


@pytest.mark.parametrize("S,lo,hi", [(4099, 0, 40), (300, 0, 90), (7, 0, 3)])
def test_slash_forms_and_sigma_kernels_agree(cuda_device, S, lo, hi):
    """Round-3 split slash (cascade over the slashed sessions only + streaming
    K03) == the round-2 group pass == the per-lane form == the host twin, bit for
    bit (scores, releases, clip records, σ_eff), on storms over a session subset
    with ragged, multi-chunk (> 16) and > 64-edge sessions; both K03 device
    kernels (stream, csr) equal the host twin."""
    vb = _vouch_batch(S, 31 + S, lo=lo, hi=hi)
    fields = list(vb.__dataclass_fields__)
    g = torch.Generator().manual_seed(S)
    sigma = torch.rand((S, 16), dtype=f64, generator=g)
    sigma[sigma < 0.05] = float("nan")
    omega = torch.rand(S, dtype=f64, generator=g)
    host = LI.sigma_eff_exact(vb, sigma, omega, 100)
    vd = vb.to("cuda")
    for k in ("stream", "csr"):
        assert torch.equal(LI.sigma_eff_exact(vd, sigma.cuda(), omega.cuda(), 100, kernel=k).cpu(), host), k
    tgt = torch.randint(0, 16, (S,), dtype=u8, generator=g)
    tgt[torch.rand(S, generator=g) < 0.6] = 255
    scores = torch.rand((S, 16), dtype=f64, generator=g)
    scores[scores < 0.1] = float("nan")
    vh = LI.VouchBatch(*[getattr(vb, f).clone() for f in fields])
    want = LI.slash(vh, tgt, omega, scores.clone(), 100, clip_cap=64, with_sigma_eff=True)
    for mode in ("split", "wave", "group", "lane"):
        for fused in (True, False):
            v = vb.to("cuda")
            got = LI.slash(v, tgt.cuda(), omega.cuda(), scores.cuda(), 100, clip_cap=64, with_sigma_eff=fused,
                           mode=mode, with_touched=True)
            torch.cuda.synchronize()
            assert torch.equal(got.touched.cpu(), torch.nonzero(want.clip_count > 0).flatten()), mode
            assert torch.equal(got.clip_count.cpu(), want.clip_count), mode
            assert torch.equal(got.scores.cpu().nan_to_num(7.0), want.scores.nan_to_num(7.0)), mode
            assert torch.equal(v.active.cpu(), vh.active) and torch.equal(v.released_us.cpu(), vh.released_us)
            n = want.clip_count.clamp(max=64)
            for s in torch.nonzero(n).flatten().tolist()[:400]:
                k = int(n[s])
                for f in ("clip_voucher", "clip_depth", "clip_before", "clip_after"):
                    assert torch.equal(getattr(got, f)[s, :k].cpu(), getattr(want, f)[s, :k]), (mode, f, s)
            if fused:
                assert torch.equal(got.sigma_eff.cpu(), want.sigma_eff), mode


@pytest.mark.parametrize("degree_hi", [6, 40])
def test_agent_exposure_segmented_and_gather(cuda_device, degree_hi):
    """K04 agent form: the segmented LDS reduction (and its > 512-entries-per-wave
    in-place walk) == the host twin bit for bit; the AgentIndex gather of the
    fused MFMA rows == a session-order sum of the host rows (no atomics)."""
    from agent_hypervisor_amd.ops.global_liability import ResidentBonds

    A = 20_000
    rb = ResidentBonds(A, 4, "cpu", seed=3)
    rng = torch.Generator().manual_seed(degree_hi)
    deg = torch.randint(0, degree_hi, (A,), generator=rng)
    E = int(deg.sum())
    rb.offsets = torch.zeros(A + 1, dtype=i64)
    rb.offsets[1:] = torch.cumsum(deg, 0)
    rb.bonded = torch.rand(E, dtype=f64, generator=rng)
    rb.active = (torch.rand(E, generator=rng) < 0.8).to(u8)
    rb.expiry = torch.where(torch.rand(E, generator=rng) < 0.2, 50, -1).to(i64)
    rb.agents, rb.edges = A, E
    host = rb.exposure(torch.empty(A, dtype=f64), now_us=100)
    for f in ("offsets", "bonded", "active", "expiry"):
        setattr(rb, f, getattr(rb, f).cuda())
    dev = rb.exposure(torch.empty(A, dtype=f64, device="cuda"), now_us=100)
    assert torch.equal(dev.cpu(), host)
    S = 3000
    vb = _vouch_batch(S, 5, lo=0, hi=20)
    sigma = torch.rand((S, 16), dtype=f64, generator=rng)
    omega = torch.rand(S, dtype=f64, generator=rng)
    members = torch.randint(0, 500, (S, 16), generator=rng)
    idx = LI.agent_index(vb, members, 500)
    _, h_ex, _ = LI.bond_fused(vb, sigma, omega, 100)
    hx = LI.agent_gather(idx, h_ex, torch.empty(500, dtype=f64))
    vd = vb.to("cuda")
    didx = LI.agent_index(vd, members.cuda(), 500)
    assert torch.equal(didx.offsets.cpu(), idx.offsets) and torch.equal(didx.index.cpu(), idx.index)
    dx = torch.empty(500, dtype=f64, device="cuda")
    _, d_ex, _ = LI.bond_fused(vd, sigma.cuda(), omega.cuda(), 100, agent_exposure=dx, agent_idx=didx)
    assert torch.equal(LI.agent_gather(didx, d_ex, torch.empty(500, dtype=f64, device="cuda")).cpu(),
                       LI.agent_gather(idx, d_ex.cpu(), torch.empty(500, dtype=f64)))
    torch.testing.assert_close(dx.cpu(), hx, rtol=1e-12, atol=1e-12)
