"""Security / ring-monitoring kernels: K16 breach window, K17 token bucket,
K18 expiry tick (reference rings/breach_detector.py, security/rate_limiter.py,
rings/elevation.py:154-165, liability/quarantine.py:147-155)."""

from __future__ import annotations

from dataclasses import dataclass
from typing import Optional

import torch

from agent_hypervisor_amd.ops._launch import launch

u8, i32, i64, f64 = torch.uint8, torch.int32, torch.int64, torch.float64


@dataclass
class BreachProfiles:
    """Ring-buffer call windows of ``n`` (agent, session) profiles."""

    ts: torch.Tensor  # i64 [n, cap]
    called: torch.Tensor  # u8 [n, cap]
    head: torch.Tensor  # i32 [n]
    count: torch.Tensor  # i32 [n]
    total: torch.Tensor  # i64 [n]
    tripped: torch.Tensor  # u8 [n]
    tripped_at_us: torch.Tensor  # i64 [n]
    ring_counts: Optional[torch.Tensor] = None  # i64 [n, 4] calls per called ring

    @classmethod
    def allocate(cls, n: int, cap: int = 1000, device="cpu", ring_counts: bool = False) -> "BreachProfiles":
        z = lambda shape, dt: torch.zeros(shape, dtype=dt, device=device)  # noqa: E731
        return cls(z((n, cap), i64), z((n, cap), u8), z(n, i32), z(n, i32), z(n, i64), z(n, u8), z(n, i64),
                   z((n, 4), i64) if ring_counts else None)

    def grow(self, n: int) -> "BreachProfiles":
        """Copy into tables of ``n`` ≥ current rows (new rows zeroed)."""
        def g(t):
            if t is None:
                return None
            out = torch.zeros((n,) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
            out[: t.shape[0]] = t
            return out
        return BreachProfiles(*(g(getattr(self, f)) for f in ("ts", "called", "head", "count", "total", "tripped",
                                                             "tripped_at_us", "ring_counts")))


def breach_record(p: BreachProfiles, now_us, agent_ring, called_ring, window_s: int = 60, cooldown_s: int = 30,
                  rows: Optional[torch.Tensor] = None, offsets: Optional[torch.Tensor] = None):
    """Record calls → (severity u8, rate f64, hits i32, event u8, window i32), one entry per call.

    Without ``rows``/``offsets`` profile ``i`` receives call ``i``.  With them,
    group ``g`` applies calls ``offsets[g]:offsets[g+1]`` in order to profile
    ``rows[g]`` (repeated calls of one profile in one launch)."""
    calls = now_us.numel()
    groups = p.head.numel() if rows is None else rows.numel()
    dev = p.head.device
    sev = torch.empty(calls, dtype=u8, device=dev)
    rate = torch.empty(calls, dtype=f64, device=dev)
    hits = torch.zeros(calls, dtype=i32, device=dev)
    ev = torch.empty(calls, dtype=u8, device=dev)
    win = torch.empty(calls, dtype=i32, device=dev)
    launch(
        "breach",
        {"n": groups, "window_cap": p.ts.shape[1], "window_us": int(window_s * 1_000_000),
         "cooldown_us": int(cooldown_s * 1_000_000)},
        dict(rows=rows, offsets=offsets, now_us=now_us, agent_ring=agent_ring, new_called=called_ring, ts=p.ts,
             called=p.called, head=p.head, count=p.count, total=p.total, tripped=p.tripped,
             tripped_at_us=p.tripped_at_us, ring_counts=p.ring_counts, severity=sev, rate=rate, hits=hits, event=ev,
             window=win),
        dict(rows=i32, offsets=i32, now_us=i64, agent_ring=u8, new_called=u8, ring_counts=i64),
    )
    return sev, rate, hits, ev, win


def token_bucket(tokens, last_us, capacity, rate, cost, now_us: int, rows=None, offsets=None, total=None,
                 rejected=None) -> torch.Tensor:
    """Lazy refill then consume (in place) → ok u8 per request.

    Without ``rows``/``offsets`` bucket ``i`` serves request ``i``; with them,
    group ``g`` serves requests ``offsets[g]:offsets[g+1]`` in order from bucket
    ``rows[g]``, counting them into ``total``/``rejected`` when given."""
    ok = torch.empty(cost.numel(), dtype=u8, device=tokens.device)
    launch(
        "bucket",
        {"n": tokens.numel() if rows is None else rows.numel(), "now_us": int(now_us)},
        dict(rows=rows, offsets=offsets, tokens=tokens, last_us=last_us, capacity=capacity, rate=rate, cost=cost,
             total=total, rejected=rejected, ok=ok),
        dict(rows=i32, offsets=i32, tokens=f64, last_us=i64, capacity=f64, rate=f64, cost=f64, total=i64,
             rejected=i64),
    )
    return ok


def expiry_tick(active, expires_us, now_us: int, released_us=None) -> torch.Tensor:
    """Deactivate records whose expiry is strictly before ``now_us`` (in place)."""
    expired = torch.empty(active.numel(), dtype=u8, device=active.device)
    launch(
        "expiry",
        {"n": active.numel(), "now_us": int(now_us)},
        dict(active=active, expires_us=expires_us, released_us=released_us, expired=expired),
        dict(active=u8, expires_us=i64, released_us=i64),
    )
    return expired
