"""Cross-rank governance views under session sharding (SURVEY §2.13, X01–X10).

Every liability invariant of the reference is session-scoped, so the per-session
pipeline needs no communication; only agent-global and job-global views do.  They
are computed here with ``torch.distributed`` (backend ``"nccl"`` = RCCL over
xGMI on MI355X, ``"gloo"`` in the CPU test harness) on an epoch cadence, never on
the per-session critical path.

=====  =====================================  ===============================
X      view                                    collective
=====  =====================================  ===============================
X01    Σ active bonded by voucher (liability)  all_reduce(SUM) over [A] fp64
X02    slash effects on agent σ                all_reduce(MIN) blacklist +
                                               all_reduce(PROD) clip factors,
                                               or sparse all_gather (id, factor)
X03    ledger risk partials                    all_reduce(SUM) fixed-point i64
X04    job counters (stats endpoint)           all_reduce(SUM) [6] i64
X05    earliest-session ring of an agent       all_reduce(MIN) packed i64 key
X06    Merkle commitments                      all_gather (slot, root, count)
X08    cache invalidation                      broadcast of agent ids
X09    latency histograms                      gather to rank 0 (all_reduce SUM)
=====  =====================================  ===============================

All functions are no-ops returning the local value when no process group is
initialised (single rank).  A thread may instead install an in-process
:class:`~agent_hypervisor_amd.parallel.fake.FakeGroup` (``fake.run_ranks``), which
runs the same merge math over simulated ranks for unit tests.
"""

from __future__ import annotations

import threading
from typing import Optional

import torch
import torch.distributed as dist

FIXED_POINT_SCALE = 1 << 40  # X03: risk partials as int64 fixed point

_thread = threading.local()


def set_thread_group(group) -> None:
    """Install (or clear, with None) this thread's in-process fake communicator."""
    _thread.group = group


def _comm():
    """The communicator of this thread: its fake group if one is installed, else
    ``torch.distributed`` (same method names for the calls used here)."""
    g = getattr(_thread, "group", None)
    return g if g is not None else dist


def _ready() -> bool:
    g = getattr(_thread, "group", None)
    if g is not None:
        return g.get_world_size() > 1
    return dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1


def world() -> int:
    return _comm().get_world_size() if _ready() else 1


def rank() -> int:
    return _comm().get_rank() if _ready() else 0


# -- X04 ----------------------------------------------------------------------------
def pipeline_stats(engine, batch=None) -> torch.Tensor:
    """Counters of the governance pipeline as int64[6] on the engine device:
    sessions, ok, participants, deltas, commitments, archived.

    When the batch was launched with a ``stats`` accumulator the kernel already
    reduced them; otherwise they are reduced from the session table rows."""
    t = engine.sessions
    s = batch.slots() if batch is not None else torch.arange(t.capacity, device=t.sess_state.device)
    st = t.sess_state.index_select(0, s)
    out = torch.stack([
        torch.tensor(s.numel(), device=st.device, dtype=torch.int64),
        (t.status.index_select(0, s) == 0).sum(),
        t.part_count.index_select(0, s).sum(),
        t.delta_count.index_select(0, s).sum(),
        (t.committed_at_us.index_select(0, s) > 0).sum(),
        (st == 4).sum(),
    ]).to(torch.int64)
    return out


def allreduce_stats(stats: torch.Tensor) -> torch.Tensor:
    if _ready():
        _comm().all_reduce(stats, op=dist.ReduceOp.SUM)
    return stats


# -- X01 ----------------------------------------------------------------------------
def allreduce_exposure(exposure: torch.Tensor) -> torch.Tensor:
    """Σ active bonded amount per voucher over every rank's sessions ([A] fp64)."""
    if _ready():
        _comm().all_reduce(exposure, op=dist.ReduceOp.SUM)
    return exposure


# -- X02 ----------------------------------------------------------------------------
#
# Merge convention.  Within one rank, slashes run in the reference order: the
# vouchee is blacklisted (σ → 0) first and its vouchers are clipped after, so an
# agent blacklisted and then clipped in the same cascade (possible only through
# a vouch cycle) ends at the floor, as SlashingEngine leaves it.  Across ranks
# (concurrent sessions, no defined order):
#   * clips commute: factors Π(1−ω) multiply and the floor is applied once —
#     exact, because max(max(x·a, F)·b, F) = max(x·a·b, F) for a, b ≤ 1;
#   * a blacklist zeroes the agent; if every rank that blacklisted it reports the
#     floor outcome (blacklist-then-clip), the merged σ is the floor.
# Each rank contributes a blacklist code per agent: 0 none, 1 ended at the floor,
# 2 ended at 0; codes merge with MAX (the lower outcome wins).


def _apply_slash(sigma: torch.Tensor, factor: torch.Tensor, touched: torch.Tensor, code: torch.Tensor,
                 floor: float) -> torch.Tensor:
    out = torch.where(touched, torch.clamp(sigma * factor, min=floor), sigma)
    out = torch.where(code == 1, torch.full_like(out, floor), out)
    return torch.where(code >= 2, torch.zeros_like(out), out)


def merge_slash_effects(
    sigma: torch.Tensor, blacklist: torch.Tensor, clip_factor: torch.Tensor, floor: float = 0.05,
    floored: Optional[torch.Tensor] = None,
) -> torch.Tensor:
    """Exact cross-rank merge of slash effects on agent σ (dense [A] form).

    ``blacklist`` is nonzero where this rank blacklisted the agent; ``floored``
    (optional) marks the blacklisted agents this rank clipped afterwards (their
    local outcome is the floor); ``clip_factor`` is the product Π(1−ω) of the
    clips this rank applied (1 where none).  See the merge convention above."""
    code = torch.where(blacklist.to(torch.bool), torch.full_like(blacklist, 2, dtype=torch.int32),
                       torch.zeros_like(blacklist, dtype=torch.int32))
    if floored is not None:
        code = torch.where(code.bool() & floored.to(torch.bool), torch.ones_like(code), code)
    cf = clip_factor.clone()
    if _ready():
        _comm().all_reduce(code, op=dist.ReduceOp.MAX)
        _comm().all_reduce(cf, op=dist.ReduceOp.PRODUCT)
    return _apply_slash(sigma, cf, cf < 1.0, code, floor)


def merge_slash_sparse(
    sigma: torch.Tensor, blacklist_ids: torch.Tensor, clip_ids: torch.Tensor, clip_factors: torch.Tensor,
    floor: float = 0.05, floored_ids: Optional[torch.Tensor] = None,
) -> torch.Tensor:
    """Sparse form of X02 for slash storms that touch few agents.

    Each rank contributes only the agents it slashed — ``blacklist_ids`` (int32),
    ``floored_ids`` (the blacklisted agents it clipped afterwards) and
    ``(clip_ids, clip_factors)`` pairs (int32, fp64 Π(1−ω), duplicates allowed) —
    instead of a dense [A] vector.  The lists are all-gathered (padded to the
    longest rank's list) and applied locally: factors PROD-scattered, blacklist
    codes MAX-scattered, one floor; identical to :func:`merge_slash_effects` on
    the densified inputs.  Returns the merged σ (``sigma`` is not modified)."""
    dev = sigma.device
    bl = blacklist_ids.to(device=dev, dtype=torch.int64).reshape(-1)
    fl = (floored_ids if floored_ids is not None else torch.empty(0)).to(device=dev, dtype=torch.int64).reshape(-1)
    ci = clip_ids.to(device=dev, dtype=torch.int64).reshape(-1)
    cf = clip_factors.to(device=dev, dtype=torch.float64).reshape(-1)
    if ci.numel() != cf.numel():
        raise ValueError("clip_ids and clip_factors must have the same length")
    # per-rank blacklist codes: 2 (zero) unless floored on this rank (1)
    bc = torch.full((bl.numel(),), 2, dtype=torch.int64, device=dev)
    if fl.numel() and bl.numel():
        bc = torch.where(torch.isin(bl, fl), torch.ones_like(bc), bc)
    if _ready():
        c = _comm()
        w = c.get_world_size()
        n = torch.tensor([bl.numel(), ci.numel()], dtype=torch.int64, device=dev)
        sizes = [torch.zeros_like(n) for _ in range(w)]
        c.all_gather(sizes, n)
        mb = max(int(t[0]) for t in sizes)
        mc = max(int(t[1]) for t in sizes)
        pb = torch.full((max(mb, 1),), -1, dtype=torch.int64, device=dev)
        pb[: bl.numel()] = bl
        pc = torch.zeros(max(mb, 1), dtype=torch.int64, device=dev)
        pc[: bc.numel()] = bc
        pi = torch.full((max(mc, 1),), -1, dtype=torch.int64, device=dev)
        pi[: ci.numel()] = ci
        pf = torch.ones(max(mc, 1), dtype=torch.float64, device=dev)
        pf[: cf.numel()] = cf
        gb = [torch.empty_like(pb) for _ in range(w)]
        gc = [torch.empty_like(pc) for _ in range(w)]
        gi = [torch.empty_like(pi) for _ in range(w)]
        gf = [torch.empty_like(pf) for _ in range(w)]
        c.all_gather(gb, pb)
        c.all_gather(gc, pc)
        c.all_gather(gi, pi)
        c.all_gather(gf, pf)
        bl, bc = torch.cat(gb), torch.cat(gc)
        keep = bl >= 0
        bl, bc = bl[keep], bc[keep]
        ci = torch.cat(gi)
        cf = torch.cat(gf)
        keep = ci >= 0
        ci, cf = ci[keep], cf[keep]
    factor = torch.ones_like(sigma, dtype=torch.float64)
    if ci.numel():
        factor.index_reduce_(0, ci, cf, "prod")
    touched = torch.zeros(sigma.numel(), dtype=torch.bool, device=dev)
    touched[ci] = True
    touched &= factor < 1.0
    code = torch.zeros(sigma.numel(), dtype=torch.int64, device=dev)
    if bl.numel():
        code.index_reduce_(0, bl, bc, "amax")
    return _apply_slash(sigma, factor, touched, code, floor)


def merge_slash_fixed(
    sigma: torch.Tensor, blacklist_ids: torch.Tensor, pair_ids: torch.Tensor, pair_factors: torch.Tensor,
    floor: float = 0.05, factor: Optional[torch.Tensor] = None, blacklist_codes: Optional[torch.Tensor] = None,
) -> torch.Tensor:
    """X02 for a slash stage inside a timed step: fixed-capacity buffers (unused
    entries id −1 / factor 1, the ``slash_clip`` kernel's output) are all-gathered
    with no size exchange and no host synchronisation, then applied sparsely by
    the ``x02_apply`` kernels (csrc/hip/global_liability.hip): only touched
    agents are read or written.  ``factor`` is a persistent all-ones [A] fp64
    scratch (allocated when omitted).  Every rank must pass buffers of the same
    capacity.  Updates ``sigma`` in place and returns it.

    Product order across duplicate (agent, factor) pairs is not fixed, so σ may
    differ from :func:`merge_slash_sparse` in the last bit where an agent is
    clipped more than once in one step.

    ``blacklist_codes`` (int32, per blacklist entry; default all 2) carries the
    blacklist-then-clip convention of :func:`merge_slash_effects`: 1 = the agent
    was clipped after its blacklist on its rank (ends at the floor), 2 = zero;
    the larger code wins across ranks."""
    from agent_hypervisor_amd.ops._launch import launch

    bl = blacklist_ids.to(torch.int32)
    pi = pair_ids.to(torch.int32)
    pf = pair_factors.to(torch.float64)
    bc = None if blacklist_codes is None else blacklist_codes.to(device=bl.device, dtype=torch.int32)
    if bc is not None and bc.numel() != bl.numel():
        raise ValueError("blacklist_codes must have one entry per blacklist id")
    if _ready():
        # one collective: the fixed-capacity buffers travel as one byte row
        c = _comm()
        w = c.get_world_size()
        nb, ni = bl.numel() * 4, pi.numel() * 4
        parts = [bl.contiguous().view(torch.uint8), pi.contiguous().view(torch.uint8),
                 pf.contiguous().view(torch.uint8)]
        if bc is not None:
            parts.append(bc.contiguous().view(torch.uint8))
        row = torch.cat(parts)
        rows = [torch.empty_like(row) for _ in range(w)]
        c.all_gather(rows, row)
        nf = pf.numel() * 8
        bl = torch.cat([r[:nb] for r in rows]).view(torch.int32)
        pi = torch.cat([r[nb:nb + ni] for r in rows]).view(torch.int32)
        pf = torch.cat([r[nb + ni:nb + ni + nf] for r in rows]).view(torch.float64)
        if bc is not None:
            bc = torch.cat([r[nb + ni + nf:] for r in rows]).view(torch.int32)
    if factor is None:
        factor = torch.ones_like(sigma)
    tensors = {"pair_id": pi, "pair_f": pf, "bl": bl, "factor": factor, "sigma": sigma}
    dtypes = {"pair_id": torch.int32, "pair_f": torch.float64, "bl": torch.int32, "factor": torch.float64,
              "sigma": torch.float64}
    if bc is not None:
        tensors["bl_code"] = bc
        dtypes["bl_code"] = torch.int32
    launch("x02_apply", {"npairs": int(pi.numel()), "nbl": int(bl.numel()), "floor": float(floor)}, tensors, dtypes)
    return sigma


# -- X03 ----------------------------------------------------------------------------
def allreduce_risk(partial_risk: torch.Tensor, counts: Optional[torch.Tensor] = None):
    """Sum per-agent ledger risk partials across ranks deterministically.

    fp64 partials are converted to int64 fixed point (2^-40 resolution) so the
    reduction is associative; the clamp to [0, 1] happens after the sum, as in
    LiabilityLedger.compute_risk_profile."""
    fx = torch.round(partial_risk * FIXED_POINT_SCALE).to(torch.int64)
    if _ready():
        _comm().all_reduce(fx, op=dist.ReduceOp.SUM)
        if counts is not None:
            _comm().all_reduce(counts, op=dist.ReduceOp.SUM)
    risk = (fx.to(torch.float64) / FIXED_POINT_SCALE).clamp(0.0, 1.0)
    return (risk, counts) if counts is not None else risk


# -- X05 ----------------------------------------------------------------------------
def earliest_ring(create_seq: torch.Tensor, ring: torch.Tensor) -> torch.Tensor:
    """Ring of each agent in its earliest-created session across ranks.

    Key = (global creation sequence << 8) | ring; the MIN key wins."""
    key = (create_seq.to(torch.int64) << 8) | ring.to(torch.int64)
    if _ready():
        _comm().all_reduce(key, op=dist.ReduceOp.MIN)
    return key & 0xFF


# -- X06 ----------------------------------------------------------------------------
def allgather_commitments(slots: torch.Tensor, roots: torch.Tensor, counts: torch.Tensor):
    """Gather every rank's (slot, 32-byte root, delta count) commitment records.

    Returns (rank, slot, root, count) tensors concatenated over ranks."""
    n = torch.tensor([slots.numel()], device=slots.device, dtype=torch.int64)
    if not _ready():
        r = torch.zeros_like(slots, dtype=torch.int32)
        return r, slots, roots, counts
    w = _comm().get_world_size()
    sizes = [torch.zeros_like(n) for _ in range(w)]
    _comm().all_gather(sizes, n)
    m = int(max(int(s.item()) for s in sizes))
    rec = torch.zeros((m, 10), dtype=torch.int32, device=slots.device)
    k = slots.numel()
    rec[:k, 0] = slots.to(torch.int32)
    rec[:k, 1] = counts.to(torch.int32)
    rec[:k, 2:] = roots.to(torch.int32)
    out = [torch.empty_like(rec) for _ in range(w)]
    _comm().all_gather(out, rec)
    ranks, sl, rt, ct = [], [], [], []
    for r, (sz, blk) in enumerate(zip(sizes, out)):
        c = int(sz.item())
        ranks.append(torch.full((c,), r, dtype=torch.int32, device=slots.device))
        sl.append(blk[:c, 0])
        ct.append(blk[:c, 1])
        rt.append(blk[:c, 2:])
    return torch.cat(ranks), torch.cat(sl), torch.cat(rt), torch.cat(ct)


# -- X08 ----------------------------------------------------------------------------
def broadcast_invalidations(agent_ids: torch.Tensor, src: int = 0) -> torch.Tensor:
    """Broadcast a list of agent ids whose cached σ must be dropped (Nexus cache)."""
    if not _ready():
        return agent_ids
    n = torch.tensor([agent_ids.numel()], dtype=torch.int64, device=agent_ids.device)
    _comm().broadcast(n, src)
    buf = agent_ids if _comm().get_rank() == src else torch.empty(int(n.item()), dtype=agent_ids.dtype,
                                                               device=agent_ids.device)
    _comm().broadcast(buf, src)
    return buf


# -- X09 ----------------------------------------------------------------------------
def reduce_histogram(hist: torch.Tensor) -> torch.Tensor:
    """Element-wise sum of per-rank latency histograms (every rank gets the total)."""
    if _ready():
        _comm().all_reduce(hist, op=dist.ReduceOp.SUM)
    return hist
