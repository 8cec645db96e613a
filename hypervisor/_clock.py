"""Host time base.

Every wall-clock read of the governance engines goes through :func:`now`, so a
test or a batched replay can pin time (``set_clock``) and the device kernels can
be handed the same instant as an int64 microsecond count (:func:`now_us`).
"""

from __future__ import annotations

from datetime import datetime, timezone
from time import time_ns as _time_ns
from typing import Callable, Optional

UTC = timezone.utc
_EPOCH = datetime(1970, 1, 1, tzinfo=UTC)

_dt_now = datetime.now
_override: Optional[Callable[[], datetime]] = None


def now() -> datetime:
    """Current UTC time (timezone-aware)."""
    if _override is not None:
        return _override()
    return _dt_now(UTC)


def set_clock(fn: Optional[Callable[[], datetime]]) -> None:
    """Install a clock override (``None`` restores the system clock)."""
    global _override
    _override = fn


def to_us(dt: datetime) -> int:
    """Microseconds since the Unix epoch of an aware datetime."""
    d = dt - _EPOCH
    return (d.days * 86400 + d.seconds) * 1_000_000 + d.microseconds


def from_us(us: int) -> datetime:
    from datetime import timedelta

    return _EPOCH + timedelta(microseconds=int(us))


def now_us() -> int:
    """``to_us(now())`` — without building a datetime when no clock is pinned
    (the device store's commands take integer µs; same CLOCK_REALTIME source)."""
    if _override is None:
        return _time_ns() // 1000
    return to_us(_override())
