"""Joint-liability kernels K03–K07 (reference liability/vouching.py,
liability/slashing.py).

A batch describes ``S`` sessions, each with ≤ 16 participants addressed by a
local index, and its vouch edges in creation order as CSR arrays
(``offsets[S+1]``, ``voucher``/``vouchee`` local indices, ``bonded`` amounts,
``active`` flags, ``expiry_us`` (-1 = none)).
"""

from __future__ import annotations

import os
from dataclasses import dataclass
from typing import Optional

import torch

from agent_hypervisor_amd.ops._launch import launch

TILE = 16
f64, u8, i32, i64 = torch.float64, torch.uint8, torch.int32, torch.int64


@dataclass
class VouchBatch:
    offsets: torch.Tensor  # i32 [S+1]
    voucher: torch.Tensor  # u8 [E]
    vouchee: torch.Tensor  # u8 [E]
    bonded: torch.Tensor  # f64 [E]
    active: torch.Tensor  # u8 [E]
    expiry_us: torch.Tensor  # i64 [E]
    released_us: torch.Tensor  # i64 [E]

    @property
    def sessions(self) -> int:
        return self.offsets.numel() - 1

    @property
    def device(self) -> torch.device:
        return self.offsets.device

    def to(self, device) -> "VouchBatch":
        return VouchBatch(*(getattr(self, f).to(device) for f in self.__dataclass_fields__))

    def clone(self) -> "VouchBatch":
        return VouchBatch(*(getattr(self, f).clone() for f in self.__dataclass_fields__))

    def _csr(self, now_us: int, **extra) -> tuple[dict, dict]:
        t = dict(offsets=self.offsets, voucher=self.voucher, vouchee=self.vouchee, bonded=self.bonded,
                 active=self.active, expiry_us=self.expiry_us, released_us=self.released_us)
        t.update(extra)
        return {"sessions": self.sessions, "now_us": int(now_us)}, t


_CSR_DT = dict(offsets=i32, voucher=u8, vouchee=u8, bonded=f64, active=u8, expiry_us=i64, released_us=i64,
               tiles=f64, sigma=f64, omega=f64, sigma_eff=f64, released=i32)


def build_tiles(vb: VouchBatch, now_us: int) -> torch.Tensor:
    """Dense [S,16,16] live-bond tiles (row voucher, col vouchee), creation-order sums."""
    tiles = torch.empty((vb.sessions, TILE, TILE), dtype=f64, device=vb.device)
    s, t = vb._csr(now_us, tiles=tiles, sigma=None, omega=None, sigma_eff=None, released=None)
    launch("build_tiles", s, t, _CSR_DT)
    return tiles


def bond_tiles(tiles: torch.Tensor, sigma: torch.Tensor, omega: torch.Tensor,
               members: "torch.Tensor | None" = None, agent_exposure: "torch.Tensor | None" = None):
    """K03/K04 on fp64 MFMA: (σ_eff [S,16], exposure [S,16], bonded_in [S,16]).

    σ_eff = min(σ + ω·Σ_voucher bonded, 1) per vouchee; exposure = Σ bonded per
    voucher.  Sums run in tile order (≤ 1-ulp-level differences from the
    creation-order reference; :func:`sigma_eff_exact` is bit-exact).

    With ``members`` (int64 [S,16] global agent ids) and ``agent_exposure``
    (f64 [A]), each participant's exposure is also added into the agent-indexed
    vector by the same kernel (the X01 input; fp64 atomics on the device, so the
    summation order across sessions is unspecified there)."""
    S = tiles.shape[0]
    out = [torch.empty((S, TILE), dtype=f64, device=tiles.device) for _ in range(3)]
    tensors = dict(tiles=tiles, sigma=sigma, omega=omega, sigma_eff=out[0], exposure=out[1], bonded_in=out[2])
    dtypes = dict(tiles=f64, sigma=f64, omega=f64)
    if members is not None:
        if agent_exposure is None or tuple(members.shape) != (S, TILE):
            raise ValueError("members must be int64 [S, 16] and come with agent_exposure")
        tensors.update(members=members, agent_exposure=agent_exposure)
        dtypes.update(members=torch.int64, agent_exposure=f64)
    launch("bond_tiles", {"sessions": S}, tensors, dtypes)
    return tuple(out)


@dataclass
class AgentIndex:
    """Resident agent-major index of a batch's voucher slots: agent ``a``'s
    entries ``index[offsets[a]:offsets[a+1]]`` are the flat (session·16 + local)
    positions where ``a`` vouches for someone, in session order.  Members that
    vouch for nobody always carry exposure 0 and are left out."""

    offsets: torch.Tensor  # i64 [A+1]
    index: torch.Tensor    # i32 [P]

    @property
    def agents(self) -> int:
        return self.offsets.numel() - 1


def agent_index(vb: VouchBatch, members: torch.Tensor, agents: int) -> AgentIndex:
    """Build the :class:`AgentIndex` of ``members`` (int64 [S,16] global ids) — once
    per bond graph (it depends on who vouches, not on which bonds are live)."""
    dev = vb.device
    counts = (vb.offsets[1:] - vb.offsets[:-1]).to(i64)
    sess = torch.repeat_interleave(torch.arange(vb.sessions, device=dev, dtype=i64), counts)
    pos = torch.unique(sess * TILE + vb.voucher.to(i64))  # sorted: session order
    ag = members.reshape(-1).to(i64)[pos]
    order = torch.argsort(ag, stable=True)
    offs = torch.zeros(agents + 1, dtype=i64, device=dev)
    offs[1:] = torch.cumsum(torch.bincount(ag, minlength=agents), 0)
    return AgentIndex(offs, pos[order].to(i32).contiguous())


def agent_gather(idx: AgentIndex, rows: torch.Tensor, out: torch.Tensor) -> torch.Tensor:
    """out[a] = Σ rows.flat[i] over agent a's entries, in session order — a
    segmented reduction (no atomics, deterministic; ``agent_exposure`` kernel)."""
    if out.dtype != f64 or out.numel() != idx.agents:
        raise ValueError("out must be fp64 [agents]")
    launch("agent_exposure", {"agents": idx.agents, "now_us": 0},
           {"offsets": idx.offsets, "bonded": rows.reshape(-1), "active": None, "expiry": None, "out": out,
            "index": idx.index},
           {"offsets": i64, "bonded": f64, "index": i32, "out": f64})
    return out


def bond_fused(vb: VouchBatch, sigma: torch.Tensor, omega: torch.Tensor, now_us: int,
               members: "torch.Tensor | None" = None, agent_exposure: "torch.Tensor | None" = None,
               bonded_in: bool = False, agent_idx: Optional[AgentIndex] = None):
    """K03/K04 straight from the CSR edges on fp64 MFMA (no dense tile):
    (σ_eff [S,16], exposure [S,16], bonded_in [S,16] or None).

    Same outputs as ``build_tiles`` + ``bond_tiles`` at a fraction of the HBM
    traffic; sums agree with the creation-order reference to ulp level.

    Agent-indexed exposure (X01 input), two forms:

    * ``agent_idx`` (an :class:`AgentIndex`): ``agent_exposure`` is *written*
      with each agent's exposure summed over its sessions in session order by a
      segmented reduction after the MFMA pass — no atomics, deterministic;
    * ``members``: the MFMA kernel *adds* each member's exposure into
      ``agent_exposure`` with fp64 atomics (order across sessions unspecified)."""
    S = vb.sessions
    dev = vb.device
    se = torch.empty((S, TILE), dtype=f64, device=dev)
    ex = torch.empty((S, TILE), dtype=f64, device=dev)
    bi = torch.empty((S, TILE), dtype=f64, device=dev) if bonded_in else None
    if members is not None and (agent_exposure is None or tuple(members.shape) != (S, TILE)):
        raise ValueError("members must be int64 [S, 16] and come with agent_exposure")
    if agent_idx is not None and (agent_exposure is None or members is not None):
        raise ValueError("agent_idx needs agent_exposure (and no members)")
    launch("bond_fused", {"sessions": S, "now_us": int(now_us)},
           dict(offsets=vb.offsets, voucher=vb.voucher, vouchee=vb.vouchee, bonded=vb.bonded, active=vb.active,
                expiry_us=vb.expiry_us, sigma=sigma, omega=omega, sigma_eff=se, exposure=ex, bonded_in=bi,
                members=members, agent_exposure=agent_exposure if members is not None else None),
           dict(_CSR_DT, exposure=f64, bonded_in=f64, members=torch.int64, agent_exposure=f64))
    if agent_idx is not None:
        agent_gather(agent_idx, ex, agent_exposure)
    return se, ex, bi


SIGMA_KERNEL = os.environ.get("AHV_SIGMA_KERNEL", "stream")
_CLIP_OFFS: dict = {}


def sigma_eff_exact(vb: VouchBatch, sigma: torch.Tensor, omega: torch.Tensor, now_us: int,
                    kernel: Optional[str] = None) -> torch.Tensor:
    """K03 creation-order path: bit-identical to VouchingEngine.compute_sigma_eff.

    ``kernel``: ``"stream"`` (default; register/DPP streaming form, every load of
    a wave's 16 sessions in flight at once) or ``"csr"`` (LDS-staged form) — the
    same additions in the same order, so the results are identical."""
    k = kernel or SIGMA_KERNEL
    if k not in ("stream", "csr"):
        raise ValueError(f"unknown sigma_eff kernel {k!r}")
    out = torch.empty((vb.sessions, TILE), dtype=f64, device=vb.device)
    s, t = vb._csr(now_us, tiles=None, sigma=sigma, omega=omega, sigma_eff=out, released=None)
    launch("sigma_eff_" + ("stream" if k == "stream" else "csr"), s, t, _CSR_DT)
    return out


def release_bonds(vb: VouchBatch, now_us: int) -> torch.Tensor:
    """K07: release every active bond of each session (in place); returns counts."""
    out = torch.empty(vb.sessions, dtype=i32, device=vb.device)
    s, t = vb._csr(now_us, tiles=None, sigma=None, omega=None, sigma_eff=None, released=out)
    launch("release_bonds", s, t, _CSR_DT)
    return out


ADMIT_OK, ADMIT_SELF, ADMIT_LOW_SIGMA, ADMIT_CYCLE, ADMIT_EXPOSURE = range(5)


def vouch_admit(
    vb: VouchBatch,
    r_offsets: torch.Tensor,
    r_voucher: torch.Tensor,
    r_vouchee: torch.Tensor,
    r_sigma: torch.Tensor,
    r_pct: torch.Tensor,
    now_us: int,
    max_exposure: float = 0.80,
) -> tuple[torch.Tensor, torch.Tensor]:
    """K05: admit vouch requests per session in order → (code u8, bonded f64)."""
    n = r_voucher.numel()
    code = torch.empty(n, dtype=u8, device=vb.device)
    bonded = torch.empty(n, dtype=f64, device=vb.device)
    launch(
        "vouch_admit",
        {"sessions": vb.sessions, "now_us": int(now_us), "max_exposure": float(max_exposure)},
        dict(e_offsets=vb.offsets, e_voucher=vb.voucher, e_vouchee=vb.vouchee, e_bonded=vb.bonded,
             e_active=vb.active, e_expiry=vb.expiry_us, r_offsets=r_offsets, r_voucher=r_voucher,
             r_vouchee=r_vouchee, r_sigma=r_sigma, r_pct=r_pct, r_bonded=bonded, code=code),
        dict(e_offsets=i32, e_voucher=u8, e_vouchee=u8, e_bonded=f64, e_active=u8, e_expiry=i64,
             r_offsets=i32, r_voucher=u8, r_vouchee=u8, r_sigma=f64, r_pct=f64),
    )
    return code, bonded


@dataclass
class SlashOutcome:
    scores: torch.Tensor  # f64 [S,16] (NaN = absent)
    clip_count: torch.Tensor  # i32 [S]
    clip_voucher: torch.Tensor  # u8 [S, cap]
    clip_depth: torch.Tensor  # u8 [S, cap]
    clip_before: torch.Tensor  # f64 [S, cap]
    clip_after: torch.Tensor  # f64 [S, cap]
    sigma_eff: Optional[torch.Tensor] = None  # f64 [S,16] post-slash σ_eff (fused K03), or None
    touched: Optional[torch.Tensor] = None  # i64 [T] sessions with ≥ 1 clip (with_touched), or None

    @property
    def truncated(self) -> torch.Tensor:
        """Sessions whose clip records exceeded the cap (records dropped, state exact)."""
        return self.clip_count > self.clip_voucher.shape[1]


def slash(
    vb: VouchBatch,
    target: torch.Tensor,
    omega: torch.Tensor,
    scores: torch.Tensor,
    now_us: int,
    clip_cap: int = 64,
    zero_records: bool = True,
    with_sigma_eff: bool = False,
    mode: Optional[str] = None,
    with_touched: bool = False,
) -> SlashOutcome:
    """K06: slash ``target[s]`` in every session (cascade ≤ 2), mutating ``vb``
    (bonds released) and ``scores`` in place, like SlashingEngine.slash.  A
    target ≥ 16 (e.g. 255) leaves that session untouched (storms over a subset).

    At most ``clip_cap`` clip *records* are kept per session (``clip_count`` holds
    the true count; :attr:`SlashOutcome.truncated` flags sessions whose records
    were cut).  The cascade itself — scores and releases — never depends on the
    cap: the walk keeps its own uncapped per-edge bytes.

    ``zero_records=False`` leaves record slots past ``clip_count[s]`` undefined
    instead of zero-filling S × clip_cap records first (18 bytes each: 180 MB
    for a 625 k-session storm with cap 16 — more HBM traffic than the slash).

    ``with_sigma_eff=True`` fuses K03 into the same pass: :attr:`SlashOutcome.sigma_eff`
    is then every session's σ_eff over its post-slash live bonds with risk weight
    ``omega`` — equal, bit for bit, to ``sigma_eff_exact(vb, scores, omega, now_us)``
    run after the slash — without a second read of the bond graph.

    ``mode`` picks the device form (all give identical results): ``"split"``
    (default: cascade over the slashed sessions only, then the streaming σ_eff
    pass), ``"wave"`` (the same split, one session per wave), ``"group"`` (one
    16-lane pass per session doing both) or ``"lane"``.

    ``with_touched=True`` also returns :attr:`SlashOutcome.touched`: the sessions
    with at least one clip, in session order (int64) — compacted on the device
    (the split cascade writes per-window segments; two small kernels place them),
    which costs one 8-byte read of the count instead of a ``torch.nonzero``."""
    S = vb.sessions
    dev = vb.device
    key = (S, int(clip_cap), str(dev))
    offs = _CLIP_OFFS.get(key)
    if offs is None:  # read-only record offsets s·cap, made once per shape (not a launch per storm)
        if len(_CLIP_OFFS) >= 8:
            _CLIP_OFFS.pop(next(iter(_CLIP_OFFS)))
        offs = _CLIP_OFFS[key] = (torch.arange(S, dtype=i32, device=dev) * clip_cap).contiguous()
    alloc = torch.zeros if zero_records else torch.empty
    out = SlashOutcome(
        scores=scores,
        clip_count=torch.empty(S, dtype=i32, device=dev),  # the kernel writes every session's count
        clip_voucher=alloc((S, clip_cap), dtype=u8, device=dev),
        clip_depth=alloc((S, clip_cap), dtype=u8, device=dev),
        clip_before=alloc((S, clip_cap), dtype=f64, device=dev),
        clip_after=alloc((S, clip_cap), dtype=f64, device=dev),
    )
    fused = {}
    if with_sigma_eff:
        out.sigma_eff = torch.empty((S, TILE), dtype=f64, device=dev)
        fused = dict(bonded=vb.bonded, sigma_eff=out.sigma_eff)
    if with_touched:
        nb = (S + 255) // 256
        tt = dict(touched_tmp=torch.empty(max(S, 1), dtype=i32, device=dev),
                  touched_blocks=torch.empty(nb, dtype=i32, device=dev),
                  touched_offsets=torch.empty(nb, dtype=i32, device=dev),
                  touched=torch.empty(max(S, 1), dtype=i64, device=dev),
                  touched_total=torch.zeros(1, dtype=i64, device=dev))
        fused.update(tt)
    launch(
        "slash",
        {"sessions": S, "now_us": int(now_us), "clip_cap": int(clip_cap),
         "mode": {None: -1, "split": 0, "group": 1, "lane": 2, "wave": 3}[mode]},
        dict(offsets=vb.offsets, voucher=vb.voucher, vouchee=vb.vouchee, active=vb.active,
             expiry_us=vb.expiry_us, released_us=vb.released_us, target=target, omega=omega, scores=scores,
             clip_offsets=offs, clip_count=out.clip_count, clip_voucher=out.clip_voucher,
             clip_depth=out.clip_depth, clip_before=out.clip_before, clip_after=out.clip_after,
             clip_walk=torch.empty(max(int(vb.voucher.numel()), 1), dtype=u8, device=dev), **fused),
        dict(target=u8, omega=f64, scores=f64, bonded=f64),
    )
    if with_touched:
        out.touched = fused["touched"][: int(fused["touched_total"].item())]
    return out


def from_engine(engine, sessions: list[str], participants: list[list[str]], device="cpu") -> VouchBatch:
    """Pack a :class:`hypervisor.liability.vouching.VouchingEngine`'s edges of the
    given sessions (with each session's participant order) into a VouchBatch."""
    offsets, vr, ve, bd, ac, ex, rel = [0], [], [], [], [], [], []
    from hypervisor._clock import to_us

    for sid, parts in zip(sessions, participants):
        idx = {d: k for k, d in enumerate(parts)}
        for v in engine._by_session.get(sid, []):
            vr.append(idx[v.voucher_did])
            ve.append(idx[v.vouchee_did])
            bd.append(v.bonded_amount)
            ac.append(1 if v.is_active else 0)
            ex.append(to_us(v.expiry) if v.expiry is not None else -1)
            rel.append(to_us(v.released_at) if v.released_at is not None else 0)
        offsets.append(len(vr))
    mk = lambda xs, dt: torch.tensor(xs, dtype=dt, device=device)  # noqa: E731
    return VouchBatch(mk(offsets, i32), mk(vr, u8), mk(ve, u8), mk(bd, f64), mk(ac, u8), mk(ex, i64), mk(rel, i64))
