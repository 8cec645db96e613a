"""Security / ring-monitoring kernels: K16 breach window, K17 token bucket,
K18 expiry tick (reference rings/breach_detector.py, security/rate_limiter.py,
rings/elevation.py:154-165, liability/quarantine.py:147-155)."""

from __future__ import annotations

from dataclasses import dataclass

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

    @classmethod
    def allocate(cls, n: int, cap: int = 1000, device="cpu") -> "BreachProfiles":
        z = lambda shape, dt: torch.zeros(shape, dtype=dt, device=device)  # noqa: E731
        return cls(z((n, cap), i64), z((n, cap), u8), z(n, i32), z(n, i32), z(n, i64), z(n, u8), z(n, i64))


def breach_record(p: BreachProfiles, now_us, agent_ring, called_ring, window_s: int = 60, cooldown_s: int = 30):
    """Record one call per profile → (severity u8, rate f64, hits i32, event u8)."""
    n = p.head.numel()
    dev = p.head.device
    sev = torch.empty(n, dtype=u8, device=dev)
    rate = torch.empty(n, dtype=f64, device=dev)
    hits = torch.zeros(n, dtype=i32, device=dev)
    ev = torch.empty(n, dtype=u8, device=dev)
    launch(
        "breach",
        {"n": n, "window_cap": p.ts.shape[1], "window_us": int(window_s * 1_000_000),
         "cooldown_us": int(cooldown_s * 1_000_000)},
        dict(now_us=now_us, agent_ring=agent_ring, new_called=called_ring, ts=p.ts, called=p.called, head=p.head,
             count=p.count, total=p.total, tripped=p.tripped, tripped_at_us=p.tripped_at_us, severity=sev,
             rate=rate, hits=hits, event=ev),
        dict(now_us=i64, agent_ring=u8, new_called=u8),
    )
    return sev, rate, hits, ev


def token_bucket(tokens, last_us, capacity, rate, cost, now_us: int) -> torch.Tensor:
    """Lazy refill then consume for every bucket (in place) → ok u8."""
    ok = torch.empty(tokens.numel(), dtype=u8, device=tokens.device)
    launch(
        "bucket",
        {"n": tokens.numel(), "now_us": int(now_us)},
        dict(tokens=tokens, last_us=last_us, capacity=capacity, rate=rate, cost=cost, ok=ok),
        dict(tokens=f64, last_us=i64, capacity=f64, rate=f64, cost=f64),
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
