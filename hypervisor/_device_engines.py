"""Device-resident variants of the stand-alone governance engines.

The reference keeps these engines as plain Python objects (dicts of dataclasses,
deques, per-call loops).  Here each one can instead hold its state as columns on
the GPU — a row per profile / bucket / record / agent — and run its hot method
as one batched kernel over a *batch of calls*:

* RingBreachDetector (reference rings/breach_detector.py:20-218) — K16
  ``breach``: ``record_calls_batch``, tensor form ``record_rows``
* AgentRateLimiter (security/rate_limiter.py:17-176) — K17 ``bucket``:
  ``check_batch``, tensor form ``check_rows``
* QuarantineManager (liability/quarantine.py:51-155) — K18 ``expiry``: ``tick``
* RingElevationManager (rings/elevation.py:60-178) — K18 ``expiry``: ``tick``
* LiabilityLedger (liability/ledger.py:50-169) — K22 ``ledger``:
  ``compute_risk_profiles``
* VectorClockManager (session/vector_clock.py:71-165) — K19 ``vclock``:
  ``apply_batch``
* IntentLockManager (session/intent_locks.py:45-196) — K20 ``locks``:
  ``acquire_batch``

The stateless batched paths — K02 ``RingEnforcer.check_batch``, K21
``CausalAttributor.attribute_batch``, K22-drift ``CMVKAdapter.record_drift_batch``
— live on the host classes themselves.

Construct one with the host class and a ``device`` — ``RingBreachDetector(
device="cuda")`` returns a :class:`DeviceRingBreachDetector` — or directly.  The
scalar API of the host engine is kept (a scalar call is a batch of one) and its
results are the host engine's results: the GPU tests replay one random call
stream through both and compare every return value, event and stat.  On
``device="cpu"`` the same code drives the kernels' host twins.

Host-side metadata that no kernel reads (DIDs, reasons, free-text details, lock
ids) stays in Python; every quantity a decision depends on — windows, tokens,
expiry/activity flags, clocks, ledger entries — lives in the device columns and
is read back only as the batch's results.
"""

from __future__ import annotations

import os
from datetime import timedelta
from typing import Iterable, Optional, Sequence

import torch

from agent_hypervisor_amd.ops import ledger as LG
from agent_hypervisor_amd.ops import security as SEC
from agent_hypervisor_amd.ops import session as SN
from hypervisor import _clock
from hypervisor._clock import now as _now
from hypervisor.liability.ledger import AgentRiskProfile, LedgerEntryType, LiabilityLedger
from hypervisor.liability.quarantine import QuarantineManager, QuarantineRecord
from hypervisor.models import ExecutionRing
from hypervisor.rings.breach_detector import BreachEvent, BreachSeverity, RingBreachDetector
from hypervisor.rings.elevation import RingElevation, RingElevationError, RingElevationManager
from hypervisor.security.rate_limiter import (
    FALLBACK_LIMIT,
    AgentRateLimiter,
    RateLimitExceeded,
    RateLimitStats,
)
from hypervisor.session.intent_locks import (
    DeadlockError,
    IntentLock,
    IntentLockManager,
    LockContentionError,
    LockIntent,
)
from hypervisor.session.vector_clock import CausalViolationError, VectorClock, VectorClockManager

i32, i64, u8, f64 = torch.int32, torch.int64, torch.uint8, torch.float64
_SEVERITY = (BreachSeverity.NONE, BreachSeverity.LOW, BreachSeverity.MEDIUM, BreachSeverity.HIGH,
             BreachSeverity.CRITICAL)


class Columns:
    """Growable device columns, one row per entity, with batched host writes.

    ``add``/``set`` queue values on the host; :meth:`flush` applies them with one
    host→device copy per touched column (before any kernel reads the table).
    :meth:`fetch` gathers rows of several columns and brings them back in one
    device→host copy.
    """

    def __init__(self, device, spec: dict, capacity: int = 256) -> None:
        self.device = torch.device(device)
        self.spec = spec  # name → (dtype, tail shape, fill)
        self.n = 0
        self.cap = max(1, capacity)
        self.t = {k: self._new(k, self.cap) for k in spec}
        self._pend: dict[str, dict[int, object]] = {}

    def _new(self, k: str, rows: int) -> torch.Tensor:
        dt, tail, fill = self.spec[k]
        return torch.full((rows,) + tuple(tail), fill, dtype=dt, device=self.device)

    def _grow(self, need: int) -> None:
        cap = max(need, 2 * self.cap)
        for k, old in self.t.items():
            new = self._new(k, cap)
            new[: self.cap] = old
            self.t[k] = new
        self.cap = cap

    def add(self, count: int = 1, **vals) -> int:
        """Append ``count`` rows (default fill, then ``vals`` on each) → first row."""
        r = self.n
        if r + count > self.cap:
            self._grow(r + count)
        self.n += count
        for k, v in vals.items():
            for j in range(count):
                self._pend.setdefault(k, {})[r + j] = v
        return r

    def set(self, row: int, **vals) -> None:
        for k, v in vals.items():
            self._pend.setdefault(k, {})[row] = v

    def flush(self) -> None:
        for k, d in self._pend.items():
            if not d:
                continue
            dt, tail, _ = self.spec[k]
            idx = torch.tensor(list(d.keys()), dtype=i64)
            val = torch.tensor(list(d.values()), dtype=dt)
            if tail:
                val = val.reshape((-1,) + tuple(tail))
            self.t[k][idx.to(self.device)] = val.to(self.device)
        self._pend.clear()

    def fetch(self, rows: Sequence[int], keys: Sequence[str]) -> dict[str, list]:
        """Values of ``keys`` at ``rows`` (one gather + one copy back)."""
        self.flush()
        if not rows:
            return {k: [] for k in keys}
        idx = torch.tensor(list(rows), dtype=i64).to(self.device)
        parts = [self.t[k][idx].reshape(len(rows), -1).to(f64) for k in keys]
        host = torch.cat(parts, dim=1).cpu()
        out, c = {}, 0
        for k, p in zip(keys, parts):
            w = p.shape[1]
            col = host[:, c:c + w]
            c += w
            dt = self.spec[k][0]
            if dt.is_floating_point:
                out[k] = col.squeeze(1).tolist() if w == 1 else col.tolist()
            else:
                out[k] = col.to(i64).squeeze(1).tolist() if w == 1 else col.to(i64).tolist()
        return out

    def __getitem__(self, k: str) -> torch.Tensor:
        return self.t[k]

    def view(self, k: str) -> torch.Tensor:
        return self.t[k][: self.n]


def _grouped(rows: Sequence[int]) -> tuple[list[int], list[int], list[int]]:
    """Stable grouping of call indices by row → (order, group rows, offsets)."""
    order = sorted(range(len(rows)), key=rows.__getitem__)
    g_rows, offs = [], []
    prev = None
    for k, i in enumerate(order):
        if rows[i] != prev:
            g_rows.append(rows[i])
            offs.append(k)
            prev = rows[i]
    offs.append(len(order))
    return order, g_rows, offs


def _upload_i64(dev: torch.device, *seqs: Sequence[int]) -> list[torch.Tensor]:
    """Several int sequences in one host→device copy (int64, split on device)."""
    flat = [x for s in seqs for x in s]
    t = torch.tensor(flat, dtype=i64).to(dev) if flat else torch.zeros(0, dtype=i64, device=dev)
    out, c = [], 0
    for s in seqs:
        out.append(t[c:c + len(s)])
        c += len(s)
    return out


# ---------------------------------------------------------------------- K16


class DeviceRingBreachDetector(RingBreachDetector):
    """Call windows as ring buffers on the device; K16 scores a batch of calls."""

    def __init__(self, window_seconds: int = 0, device="cuda", capacity: int = 256, window_cap: int = 1000) -> None:
        super().__init__(window_seconds)
        self.device = torch.device(device)
        self.window_cap = window_cap
        self._rows: dict[str, int] = {}
        self._who: list[tuple[str, str]] = []
        self.cols = Columns(self.device, {
            "ts": (i64, (window_cap,), 0), "called": (u8, (window_cap,), 0), "head": (i32, (), 0),
            "count": (i32, (), 0), "total": (i64, (), 0), "tripped": (u8, (), 0), "tripped_at_us": (i64, (), 0),
            "ring_counts": (i64, (4,), 0),
        }, capacity)

    def _row(self, agent_did: str, session_id: str, create: bool = True) -> Optional[int]:
        key = f"{agent_did}:{session_id}"
        r = self._rows.get(key)
        if r is None and create:
            r = self._rows[key] = self.cols.add()
            self._who.append((agent_did, session_id))
        return r

    def _profiles_view(self) -> SEC.BreachProfiles:
        c = self.cols
        return SEC.BreachProfiles(c["ts"], c["called"], c["head"], c["count"], c["total"], c["tripped"],
                                  c["tripped_at_us"], c["ring_counts"])

    def record_calls_batch(self, calls: Iterable[tuple], now=None) -> list[Optional[BreachEvent]]:
        """Record ``(agent_did, session_id, agent_ring, called_ring)`` calls at one
        instant → the BreachEvent (or None) of each call, as sequential
        :meth:`record_call` would return them; events join the history in call order."""
        calls = list(calls)
        if not calls:
            return []
        t = now or _now()
        rows = [self._row(a, s) for a, s, _, _ in calls]
        order, g_rows, offs = _grouped(rows)
        self.cols.flush()
        dev = self.device
        gr, go, ar, cr = _upload_i64(dev, g_rows, offs, [int(calls[i][2].value) for i in order],
                                     [int(calls[i][3].value) for i in order])
        now_t = torch.full((len(calls),), _clock.to_us(t), dtype=i64, device=dev)
        sev, rate, hits, ev, win = SEC.breach_record(
            self._profiles_view(), now_t, ar.to(u8), cr.to(u8), self.window_seconds, self.CIRCUIT_BREAKER_COOLDOWN,
            rows=gr.to(i32), offsets=go.to(i32))
        host = torch.stack([sev.to(f64), rate, hits.to(f64), ev.to(f64), win.to(f64)]).cpu().tolist()
        out: list[Optional[BreachEvent]] = [None] * len(calls)
        for k, i in enumerate(order):
            if not host[3][k]:
                continue
            a, s = calls[i][0], calls[i][1]
            h, w, r = int(host[2][k]), int(host[4][k]), host[1][k]
            out[i] = BreachEvent(
                agent_did=a, session_id=s, severity=_SEVERITY[int(host[0][k])], anomaly_score=r,
                call_count_window=w, expected_rate=0.0, actual_rate=r, timestamp=t,
                details=f"{h}/{w} calls to more-privileged rings in {self.window_seconds}s window")
        self._breach_history.extend(e for e in out if e is not None)
        return out

    def rows_for(self, keys: Sequence[tuple[str, str]]) -> torch.Tensor:
        """Device rows (int32) of ``(agent_did, session_id)`` profiles, interning new ones."""
        rows = [self._row(a, s) for a, s in keys]
        self.cols.flush()
        return torch.tensor(rows, dtype=i32).to(self.device)

    def record_rows(self, rows: torch.Tensor, agent_ring: torch.Tensor, called_ring: torch.Tensor,
                    now=None) -> dict[str, torch.Tensor]:
        """Tensor form of :meth:`record_calls_batch` for calls already on the
        device (int32 profile rows from :meth:`rows_for`, uint8 rings): grouping
        by profile is a stable device sort; the per-call outputs come back in call
        order as device tensors, and only the (rare) breach events are copied to
        the host to join the history."""
        t = now or _now()
        n = rows.numel()
        order = torch.sort(rows, stable=True).indices
        srows = rows[order]
        g_rows, counts = torch.unique_consecutive(srows, return_counts=True)
        offs = torch.zeros(g_rows.numel() + 1, dtype=i32, device=rows.device)
        offs[1:] = counts.cumsum(0)
        now_t = torch.full((n,), _clock.to_us(t), dtype=i64, device=rows.device)
        sev, rate, hits, ev, win = SEC.breach_record(
            self._profiles_view(), now_t, agent_ring[order].contiguous(), called_ring[order].contiguous(),
            self.window_seconds, self.CIRCUIT_BREAKER_COOLDOWN, rows=g_rows.to(i32), offsets=offs)
        out = {}
        for k, v in (("severity", sev), ("rate", rate), ("hits", hits), ("event", ev), ("window", win)):
            o = torch.empty_like(v)
            o[order] = v
            out[k] = o
        idx = torch.nonzero(out["event"]).flatten()
        if idx.numel():
            host = torch.stack([idx.to(f64), out["severity"][idx].to(f64), out["rate"][idx], out["hits"][idx].to(f64),
                                out["window"][idx].to(f64), rows[idx].to(f64)]).cpu().tolist()
            for i, sv, r, h, w, row in zip(*host):
                a, s = self._who[int(row)]
                self._breach_history.append(BreachEvent(
                    agent_did=a, session_id=s, severity=_SEVERITY[int(sv)], anomaly_score=r,
                    call_count_window=int(w), expected_rate=0.0, actual_rate=r, timestamp=t,
                    details=f"{int(h)}/{int(w)} calls to more-privileged rings in {self.window_seconds}s window"))
        return out

    def record_call(self, agent_did, session_id, agent_ring, called_ring) -> Optional[BreachEvent]:
        return self.record_calls_batch([(agent_did, session_id, agent_ring, called_ring)])[0]

    def is_breaker_tripped(self, agent_did: str, session_id: str) -> bool:
        r = self._row(agent_did, session_id, create=False)
        if r is None:
            return False
        v = self.cols.fetch([r], ["tripped", "tripped_at_us"])
        if not v["tripped"][0]:
            return False
        at = v["tripped_at_us"][0]
        cool_end = at + self.CIRCUIT_BREAKER_COOLDOWN * 1_000_000
        if at != 0 and not _clock.now_us() < cool_end:
            self.cols.set(r, tripped=0)
            return False
        return True

    def reset_breaker(self, agent_did: str, session_id: str) -> None:
        r = self._row(agent_did, session_id, create=False)
        if r is not None:
            self.cols.set(r, tripped=0, tripped_at_us=0)

    def get_agent_stats(self, agent_did: str, session_id: str) -> dict:
        r = self._row(agent_did, session_id, create=False)
        if r is None:
            return {"total_calls": 0, "window_calls": 0, "breaker_tripped": False}
        v = self.cols.fetch([r], ["total", "count", "tripped", "ring_counts"])
        return {
            "total_calls": v["total"][0],
            "window_calls": v["count"][0],
            "breaker_tripped": bool(v["tripped"][0]),
            "ring_distribution": {ring: c for ring, c in enumerate(v["ring_counts"][0]) if c},
        }


# ---------------------------------------------------------------------- K17


class DeviceAgentRateLimiter(AgentRateLimiter):
    """Token buckets as device columns; K17 serves a batch of requests."""

    def __init__(self, ring_limits=None, device="cuda", capacity: int = 256) -> None:
        super().__init__(ring_limits)
        self.device = torch.device(device)
        self._rows: dict[str, int] = {}
        self._meta: list[list] = []  # row → [agent_did, ring, has_stats]
        self.cols = Columns(self.device, {
            "tokens": (f64, (), 0.0), "last_us": (i64, (), 0), "capacity": (f64, (), 0.0), "rate": (f64, (), 0.0),
            "total": (i64, (), 0), "rejected": (i64, (), 0),
        }, capacity)

    def _fill(self, row: int, ring: ExecutionRing, t_us: int) -> None:
        rate, cap = self._limits.get(ring, FALLBACK_LIMIT)
        self.cols.set(row, tokens=float(cap), last_us=t_us, capacity=float(cap), rate=float(rate))

    def _row(self, agent_did: str, session_id: str, ring: ExecutionRing, t_us: int) -> int:
        key = f"{agent_did}:{session_id}"
        r = self._rows.get(key)
        if r is None:
            r = self._rows[key] = self.cols.add()
            self._meta.append([agent_did, ring, False])
            self._fill(r, ring, t_us)
        return r

    def check_batch(self, requests: Iterable[tuple], now=None) -> list[bool]:
        """Serve ``(agent_did, session_id, ring[, cost])`` requests at one instant →
        admitted flags, as sequential :meth:`try_check` calls would return them."""
        reqs = list(requests)
        if not reqs:
            return []
        t_us = _clock.to_us(now or _now())
        rows = []
        for q in reqs:
            r = self._row(q[0], q[1], q[2], t_us)
            if not self._meta[r][2]:
                self._meta[r][2] = True
                self._meta[r][1] = q[2]
            rows.append(r)
        order, g_rows, offs = _grouped(rows)
        self.cols.flush()
        dev = self.device
        gr, go = _upload_i64(dev, g_rows, offs)
        cost = torch.tensor([float(reqs[i][3]) if len(reqs[i]) > 3 else 1.0 for i in order], dtype=f64).to(dev)
        c = self.cols
        ok = SEC.token_bucket(c["tokens"], c["last_us"], c["capacity"], c["rate"], cost, t_us, rows=gr.to(i32),
                              offsets=go.to(i32), total=c["total"], rejected=c["rejected"]).cpu().tolist()
        out = [False] * len(reqs)
        for k, i in enumerate(order):
            out[i] = bool(ok[k])
        return out

    def rows_for(self, keys: Sequence[tuple[str, str, ExecutionRing]]) -> torch.Tensor:
        """Device rows (int32) of ``(agent_did, session_id, ring)`` buckets, creating new ones."""
        t_us = _clock.now_us()
        rows = []
        for a, s, ring in keys:
            r = self._row(a, s, ring, t_us)
            if not self._meta[r][2]:
                self._meta[r][2] = True
                self._meta[r][1] = ring
            rows.append(r)
        self.cols.flush()
        return torch.tensor(rows, dtype=i32).to(self.device)

    def check_rows(self, rows: torch.Tensor, cost: Optional[torch.Tensor] = None, now=None) -> torch.Tensor:
        """Tensor form of :meth:`check_batch` (rows from :meth:`rows_for`) → admitted
        flags (uint8, call order) on the device."""
        t_us = _clock.to_us(now or _now())
        n = rows.numel()
        order = torch.sort(rows, stable=True).indices
        g_rows, counts = torch.unique_consecutive(rows[order], return_counts=True)
        offs = torch.zeros(g_rows.numel() + 1, dtype=i32, device=rows.device)
        offs[1:] = counts.cumsum(0)
        cost_s = (torch.ones(n, dtype=f64, device=rows.device) if cost is None else cost[order].to(f64)).contiguous()
        c = self.cols
        ok_s = SEC.token_bucket(c["tokens"], c["last_us"], c["capacity"], c["rate"], cost_s, t_us,
                                rows=g_rows.to(i32), offsets=offs, total=c["total"], rejected=c["rejected"])
        ok = torch.empty_like(ok_s)
        ok[order] = ok_s
        return ok

    def check(self, agent_did, session_id, ring, cost: float = 1.0) -> bool:
        if self.check_batch([(agent_did, session_id, ring, cost)])[0]:
            return True
        r = self._rows[f"{agent_did}:{session_id}"]
        n = self.cols.fetch([r], ["rejected"])["rejected"][0]
        raise RateLimitExceeded(f"Agent {agent_did} exceeded rate limit for ring {ring.value} ({n} rejections)")

    def try_check(self, agent_did, session_id, ring, cost: float = 1.0) -> bool:
        return self.check_batch([(agent_did, session_id, ring, cost)])[0]

    def update_ring(self, agent_did, session_id, new_ring) -> None:
        t_us = _clock.now_us()
        key = f"{agent_did}:{session_id}"
        r = self._rows.get(key)
        if r is None:
            self._row(agent_did, session_id, new_ring, t_us)
            return
        self._fill(r, new_ring, t_us)
        if self._meta[r][2]:
            self._meta[r][1] = new_ring

    def get_stats(self, agent_did, session_id) -> Optional[RateLimitStats]:
        r = self._rows.get(f"{agent_did}:{session_id}")
        if r is None or not self._meta[r][2]:
            return None
        # lazy refill at "now" (cost 0 admits and consumes nothing), as TokenBucket.available
        self.cols.flush()
        c = self.cols
        rr = torch.tensor([r], dtype=i32).to(self.device)
        SEC.token_bucket(c["tokens"], c["last_us"], c["capacity"], c["rate"], torch.zeros(1, dtype=f64,
                         device=self.device), _clock.now_us(), rows=rr, offsets=torch.tensor([0, 1], dtype=i32,
                         device=self.device))
        v = c.fetch([r], ["total", "rejected", "tokens", "capacity"])
        return RateLimitStats(agent_did=self._meta[r][0], ring=self._meta[r][1], total_requests=v["total"][0],
                              rejected_requests=v["rejected"][0], tokens_available=v["tokens"][0],
                              capacity=v["capacity"][0])

    @property
    def tracked_agents(self) -> int:
        return len(self._rows)


# ---------------------------------------------------------------------- K18


class _ExpiryRows:
    """active / expires_us / released_us columns of expiring records (K18)."""

    def __init__(self, device, capacity: int) -> None:
        self.cols = Columns(device, {"active": (u8, (), 0), "expires_us": (i64, (), -1),
                                     "released_us": (i64, (), 0)}, capacity)

    def add(self, expires_us: int) -> int:
        return self.cols.add(active=1, expires_us=expires_us)

    def deactivate(self, row: int, released_us: int = 0) -> None:
        self.cols.set(row, active=0, released_us=released_us)

    def tick(self, now_us: int) -> list[int]:
        c = self.cols
        c.flush()
        if c.n == 0:
            return []
        expired = SEC.expiry_tick(c.view("active"), c.view("expires_us"), now_us, c.view("released_us"))
        return torch.nonzero(expired).flatten().cpu().tolist()


class DeviceQuarantineManager(QuarantineManager):
    """Quarantine records' activity/expiry on the device; K18 ticks all of them."""

    def __init__(self, device="cuda", capacity: int = 256) -> None:
        super().__init__()
        self.device = torch.device(device)
        self._exp = _ExpiryRows(self.device, capacity)
        self._recs: list[QuarantineRecord] = []  # row → record (metadata view)
        self._row_of: dict[str, int] = {}

    def quarantine(self, agent_did, session_id, reason, details: str = "", duration_seconds=None,
                   forensic_data=None) -> QuarantineRecord:
        return self.quarantine_batch([(agent_did, session_id, reason, details, duration_seconds, forensic_data)])[0]

    def quarantine_batch(self, requests: Iterable[tuple]) -> list[QuarantineRecord]:
        """Quarantine ``(agent_did, session_id, reason[, details, duration_seconds,
        forensic_data])`` in order; rows are written to the device in one flush."""
        out = []
        for q in requests:
            agent, session, reason = q[0], q[1], q[2]
            details = q[3] if len(q) > 3 else ""
            secs_in = q[4] if len(q) > 4 else None
            forensic = q[5] if len(q) > 5 else None
            live = self.get_active_quarantine(agent, session)
            if live is not None:
                live.details += f"; escalated: {details}"
                if forensic:
                    live.forensic_data.update(forensic)
                out.append(live)
                continue
            secs = secs_in or self.DEFAULT_QUARANTINE_SECONDS
            t = _now()
            rec = QuarantineRecord(agent_did=agent, session_id=session, reason=reason, details=details, entered_at=t,
                                   expires_at=t + timedelta(seconds=secs) if secs else None,
                                   forensic_data=forensic or {})
            row = self._exp.add(_clock.to_us(rec.expires_at) if rec.expires_at is not None else -1)
            self._quarantines[rec.quarantine_id] = rec
            self._recs.append(rec)
            self._row_of[rec.quarantine_id] = row
            out.append(rec)
        self._exp.cols.flush()
        return out

    def release(self, agent_did, session_id) -> Optional[QuarantineRecord]:
        rec = self.get_active_quarantine(agent_did, session_id)
        if rec is not None:
            rec.is_active = False
            rec.released_at = _now()
            self._exp.deactivate(self._row_of[rec.quarantine_id], _clock.to_us(rec.released_at))
        return rec

    def tick(self) -> list[QuarantineRecord]:
        t = _now()
        out = []
        for r in self._exp.tick(_clock.to_us(t)):
            rec = self._recs[r]
            rec.is_active = False
            rec.released_at = t
            out.append(rec)
        return out


class DeviceRingElevationManager(RingElevationManager):
    """Elevations' activity/expiry on the device; K18 ticks all of them."""

    def __init__(self, device="cuda", capacity: int = 256) -> None:
        super().__init__()
        self.device = torch.device(device)
        self._exp = _ExpiryRows(self.device, capacity)
        self._recs: list[RingElevation] = []
        self._row_of: dict[str, int] = {}

    def request_elevation(self, agent_did, session_id, current_ring, target_ring, ttl_seconds: int = 0,
                          attestation=None, reason: str = "") -> RingElevation:
        res = self.request_elevation_batch([(agent_did, session_id, current_ring, target_ring, ttl_seconds,
                                             attestation, reason)])[0]
        if isinstance(res, Exception):
            raise res
        return res

    def request_elevation_batch(self, requests: Iterable[tuple]) -> list:
        """Grant ``(agent_did, session_id, current_ring, target_ring[, ttl, attestation,
        reason])`` requests in order → RingElevation or the RingElevationError."""
        out = []
        for q in requests:
            try:
                e = RingElevationManager.request_elevation(self, *q)
            except RingElevationError as err:
                out.append(err)
                continue
            self._row_of[e.elevation_id] = self._exp.add(_clock.to_us(e.expires_at))
            self._recs.append(e)
            out.append(e)
        self._exp.cols.flush()
        return out

    def revoke_elevation(self, elevation_id: str) -> None:
        super().revoke_elevation(elevation_id)
        self._exp.deactivate(self._row_of[elevation_id])

    def tick(self) -> list[RingElevation]:
        out = []
        for r in self._exp.tick(_clock.now_us()):
            e = self._recs[r]
            e.is_active = False
            out.append(e)
        return out


# ---------------------------------------------------------------------- K22


_LEDGER_CODE = {t: LG.LEDGER_CODE[t.value] for t in LedgerEntryType}


class DeviceLiabilityLedger(LiabilityLedger):
    """Ledger entries as a device log (agent, type, severity); K22 scores agents."""

    def __init__(self, device="cuda", capacity: int = 1024) -> None:
        super().__init__()
        self.device = torch.device(device)
        self.log = Columns(self.device, {"agent": (i32, (), 0), "type": (u8, (), 0), "severity": (f64, (), 0.0)},
                           capacity)
        self._agent_row: dict[str, int] = {}

    def record(self, agent_did, entry_type, session_id: str = "", severity: float = 0.0, details: str = "",
               related_agent=None):
        e = super().record(agent_did, entry_type, session_id, severity, details, related_agent)
        a = self._agent_row.setdefault(agent_did, len(self._agent_row))
        self.log.add(agent=a, type=_LEDGER_CODE[LedgerEntryType(entry_type)], severity=float(severity))
        return e

    def partials(self, agent_dids: Sequence[str]) -> dict[str, torch.Tensor]:
        """Per-agent ledger partials on the device (one K22 launch over the log):
        raw (unclamped) risk, slash / quarantine / clean / fault counts, fault
        severity sum and entry count — the additive state the sharded ledger
        all-reduces (X03).  Agents without entries get zeros."""
        self.log.flush()
        n, A = self.log.n, len(self._agent_row)
        dev = self.device
        rows = torch.tensor([self._agent_row.get(a, -1) for a in agent_dids], dtype=i64).to(dev)
        z = {k: torch.zeros(len(agent_dids), dtype=f64 if k in ("raw", "fault_sum") else i64, device=dev)
             for k in ("raw", "slash", "quarantine", "clean", "fault_sum", "fault_n", "total")}
        if n == 0 or A == 0:
            return z
        agent = self.log.view("agent")
        order = torch.sort(agent, stable=True).indices
        offs = torch.zeros(A + 1, dtype=i64, device=dev)
        offs[1:] = torch.bincount(agent.to(i64), minlength=A).cumsum(0)
        types = self.log.view("type")[order].contiguous()
        sev = self.log.view("severity")[order].contiguous()
        out = LG.risk_profiles(offs.to(i32), types, sev)
        fault = (self.log.view("type") == LG.LEDGER_CODE["fault_attributed"])
        fault_n = torch.bincount(agent.to(i64), weights=fault.to(f64), minlength=A).round().to(i64)
        have = rows >= 0
        r = rows.clamp(min=0)
        pick = lambda t, dt: torch.where(have, t[r].to(dt), torch.zeros((), dtype=dt, device=dev))  # noqa: E731
        z["raw"] = pick(out["raw_risk"], f64)
        z["slash"] = pick(out["slash_count"], i64)
        z["quarantine"] = pick(out["quarantine_count"], i64)
        z["clean"] = pick(out["clean_count"], i64)
        z["fault_n"] = pick(fault_n, i64)
        z["fault_sum"] = pick(out["fault_avg"], f64) * z["fault_n"].to(f64)
        z["total"] = pick(offs[1:] - offs[:-1], i64)
        return z

    def compute_risk_profiles(self, agent_dids: Sequence[str]) -> list[AgentRiskProfile]:
        """Risk profiles of many agents from one K22 launch over the whole log."""
        self.log.flush()
        n, A = self.log.n, len(self._agent_row)
        rows = [self._agent_row.get(a, -1) for a in agent_dids]
        if n == 0 or all(r < 0 for r in rows):
            return [AgentRiskProfile(agent_did=a, recommendation="admit") for a in agent_dids]
        agent = self.log.view("agent")
        order = torch.sort(agent, stable=True).indices
        offs = torch.zeros(A + 1, dtype=i64, device=self.device)
        offs[1:] = torch.bincount(agent.to(i64), minlength=A).cumsum(0)
        out = LG.risk_profiles(offs.to(i32), self.log.view("type")[order].contiguous(),
                               self.log.view("severity")[order].contiguous())
        live = [r for r in rows if r >= 0]
        idx = torch.tensor(live, dtype=i64).to(self.device)
        keys = ("risk", "recommendation", "slash_count", "quarantine_count", "clean_count", "fault_avg")
        host = torch.stack([out[k][idx].to(f64) for k in keys] + [(offs[idx + 1] - offs[idx]).to(f64)]).cpu()
        host = host.tolist()
        res, j = [], 0
        for a, r in zip(agent_dids, rows):
            if r < 0:
                res.append(AgentRiskProfile(agent_did=a, recommendation="admit"))
                continue
            risk, rec, sc, qc, cc, fa, total = (host[k][j] for k in range(7))
            j += 1
            res.append(AgentRiskProfile(
                agent_did=a, total_entries=int(total), slash_count=int(sc), quarantine_count=int(qc),
                clean_session_count=int(cc), fault_score_avg=round(fa, 4), risk_score=round(risk, 4),
                recommendation=LG.RECOMMENDATION[int(rec)]))
        return res

    def compute_risk_profile(self, agent_did: str) -> AgentRiskProfile:
        return self.compute_risk_profiles([agent_did])[0]


# ---------------------------------------------------------------------- K19


class DeviceVectorClockManager(VectorClockManager):
    """Dense clocks on the device — one component per agent (≤ 64, one lane of
    a wave each); K19 applies a batch of reads/writes in order."""

    MAX_AGENTS = 64

    def __init__(self, device="cuda", capacity: int = 256) -> None:
        super().__init__()
        self.device = torch.device(device)
        A = self.MAX_AGENTS
        self.paths = Columns(self.device, {"clock": (i32, (A,), 0)}, capacity)
        self.agents = Columns(self.device, {"clock": (i32, (A,), 0)}, A)
        self.agents.add(A)
        self._path_row: dict[str, int] = {}
        self._col: dict[str, int] = {}
        self._written: set[str] = set()

    def _agent(self, did: str) -> int:
        c = self._col.get(did)
        if c is None:
            if len(self._col) >= self.MAX_AGENTS:
                raise ValueError(f"device vector clocks hold at most {self.MAX_AGENTS} agents")
            c = self._col[did] = len(self._col)
        return c

    def _path(self, path: str) -> int:
        r = self._path_row.get(path)
        if r is None:
            r = self._path_row[path] = self.paths.add()
        return r

    def _clock_of(self, cols: Columns, row: int) -> VectorClock:
        v = cols.fetch([row], ["clock"])["clock"][0]
        names = {c: a for a, c in self._col.items()}
        return VectorClock(clocks={names[j]: int(x) for j, x in enumerate(v) if x})

    def apply_batch(self, ops: Iterable[tuple], strict: bool = True) -> list[bool]:
        """Apply ``("read"|"write", path, agent_did)`` operations in order (one
        wave, one launch) → ok flags (False = write rejected as causally stale)."""
        ops = list(ops)
        if not ops:
            return []
        codes = [SN.WRITE if o[0] == "write" else SN.READ for o in ops]
        prow = [self._path(o[1]) for o in ops]
        acol = [self._agent(o[2]) for o in ops]
        self.paths.flush()
        dev = self.device
        offs, op, pr, ac = _upload_i64(dev, [0, len(ops)], codes, prow, acol)
        ac32 = ac.to(i32)
        ok = SN.vector_clock_ops(offs.to(i32), op.to(u8), pr.to(i32), ac32, ac32, self.paths["clock"],
                                 self.agents["clock"], strict).cpu().tolist()
        for o, k in zip(ops, ok):
            if o[0] == "write":
                if k:
                    self._written.add(o[1])
                else:
                    self._conflict_count += 1
        return [bool(k) for k in ok]

    def read(self, path: str, agent_did: str) -> VectorClock:
        self.apply_batch([("read", path, agent_did)])
        return self.get_path_clock(path)

    def write(self, path: str, agent_did: str, strict: bool = True) -> VectorClock:
        if not self.apply_batch([("write", path, agent_did)], strict)[0]:
            ac, pc = self.get_agent_clock(agent_did), self.get_path_clock(path)
            raise CausalViolationError(
                f"Agent {agent_did} has stale state for {path}. "
                f"Agent clock: {ac.clocks}, Path clock: {pc.clocks}. "
                "Must re-read before writing.")
        return self.get_path_clock(path)

    def get_path_clock(self, path: str) -> VectorClock:
        r = self._path_row.get(path)
        return VectorClock() if r is None else self._clock_of(self.paths, r)

    def get_agent_clock(self, agent_did: str) -> VectorClock:
        c = self._col.get(agent_did)
        return VectorClock() if c is None else self._clock_of(self.agents, c)

    @property
    def tracked_paths(self) -> int:
        return len(self._written)


# ---------------------------------------------------------------------- K20


class DeviceIntentLockManager(IntentLockManager):
    """Intent locks whose contention decisions run on the device (K20 grant pass).

    The device keeps a resident holder table per resource — active READ and
    WRITE/EXCLUSIVE lock counts and up to 16 holder slots (agent, its reads,
    its writes) — and a batch of acquires is decided in one launch: requests
    are grouped by resource (stable, so request order holds within a resource)
    and one lane per resource walks its requests, granting or refusing each
    exactly as a sequential :meth:`acquire` would and recording the grants.
    The host keeps the lock records (ids, saga-step links, the per-resource
    index that release and the queries use) and the wait-for graph: refused
    requests take the host path, which builds the same LockContentionError /
    DeadlockError (and wait edges) sequential acquire raises.  Releases mark
    their resource stale; its row is rebuilt from the records before the next
    batch.  More than 16 concurrent holders can only be readers: the counts
    stay exact, the extra readers are granted by the host path.

    :meth:`acquire_rows` / :meth:`release_rows` are the tensor-native form
    (device tensors in, granted mask out, holds tracked only on the device)."""

    def __init__(self, record_waits: bool = False, device="cuda") -> None:
        super().__init__(record_waits)
        self.device = torch.device(device)
        self._agent_id: dict[str, int] = {}
        self._res_id: dict[str, int] = {}
        self._res_path: list[str] = []
        self._table = self._fresh(1024)
        self._dirty: set[str] = set()

    def _fresh(self, n: int) -> torch.Tensor:
        t = torch.zeros((n, SN.LOCK_ROW), dtype=i32, device=self.device)
        t[:, 2::2] = -1
        return t

    def _aid(self, did: str) -> int:
        return self._agent_id.setdefault(did, len(self._agent_id))

    def _rid(self, path: str) -> int:
        r = self._res_id.get(path)
        if r is None:
            r = self._res_id[path] = len(self._res_path)
            self._res_path.append(path)
        return r

    def release(self, lock_id: str) -> None:
        lock = self._locks.get(lock_id)
        super().release(lock_id)
        if lock is not None:
            self._dirty.add(lock.resource_path)

    def _row_of(self, path: str) -> list[int]:
        rc = wc = 0
        slots: dict[int, list[int]] = {}
        for lk in self.get_resource_locks(path):
            a = self._aid(lk.agent_did)
            w = not (lk.intent is LockIntent.READ or lk.intent == "read")
            wc += w
            rc += not w
            if a in slots or len(slots) < SN.LOCK_HOLDERS:
                c = slots.setdefault(a, [0, 0])
                c[w] += 1
        row = [rc, wc]
        for a, (r, w) in slots.items():
            row += [a, r | (w << 16)]
        row += [-1, 0] * (SN.LOCK_HOLDERS - len(slots))
        return row

    def _sync(self) -> None:
        """Grow the table to every known resource and rebuild the rows the host
        changed (releases, overflow grants) from the lock records."""
        R = len(self._res_path)
        if R > self._table.shape[0]:
            cap = self._table.shape[0]
            while cap < R:
                cap *= 2
            grown = self._fresh(cap)
            grown[: self._table.shape[0]] = self._table
            self._table = grown
        if not self._dirty:
            return
        rows, vals = [], []
        for path in self._dirty:
            r = self._res_id.get(path)
            if r is not None:
                rows.append(r)
                vals.append(self._row_of(path))
        self._dirty.clear()
        if rows:
            self._table[torch.tensor(rows, dtype=i64, device=self.device)] = \
                torch.tensor(vals, dtype=i32).to(self.device)

    def acquire(self, agent_did, session_id, resource_path, intent, saga_step_id=None) -> IntentLock:
        res = self.acquire_batch([(agent_did, session_id, resource_path, intent, saga_step_id)])[0]
        if isinstance(res, Exception):
            raise res
        return res

    def _grant(self, rs, ag, it) -> "np.ndarray":
        import numpy as np

        n = len(rs)
        order = np.argsort(rs, kind="stable").astype(np.int32)
        sr = rs[order]
        starts = np.flatnonzero(np.r_[True, sr[1:] != sr[:-1]]).astype(np.int32)
        G = len(starts)
        buf = torch.from_numpy(np.concatenate([np.r_[starts, n].astype(np.int32), order, rs, ag, it]))
        buf = buf.to(self.device)
        granted = torch.empty(n, dtype=u8, device=self.device)
        o = G + 1
        SN.lock_grant(buf[:o], buf[o: o + n], buf[o + n: o + 2 * n], buf[o + 2 * n: o + 3 * n],
                      buf[o + 3 * n:].to(u8), self._table, granted)
        return granted.cpu().numpy()

    def acquire_batch(self, requests: Iterable[tuple]) -> list:
        """``(agent_did, session_id, resource_path, intent[, saga_step_id])`` →
        IntentLock, or the LockContentionError / DeadlockError sequential
        acquire would raise, per request."""
        import numpy as np

        reqs = requests if isinstance(requests, list) else list(requests)
        n = len(reqs)
        if not n:
            return []
        aid, rid = self._aid, self._rid
        codes = SN.LOCK_INTENT
        ag = np.fromiter((aid(q[0]) for q in reqs), dtype=np.int32, count=n)
        rs = np.fromiter((rid(q[2]) for q in reqs), dtype=np.int32, count=n)
        it = np.fromiter((codes[q[3]] for q in reqs), dtype=np.int32, count=n)
        self._sync()
        ok = self._grant(rs, ag, it)
        # lock records for the grants (one timestamp per batch, ids minted in bulk), errors for the rest
        when = _now()
        hexes = os.urandom(4 * n).hex()
        locks, index = self._locks, self._resource_locks
        new = object.__new__
        out: list = [None] * n
        for i in range(n):
            q = reqs[i]
            if ok[i] == 1:
                lock = new(IntentLock)
                lid = "lock:" + hexes[8 * i: 8 * i + 8]
                lock.__dict__.update(lock_id=lid, agent_did=q[0], session_id=q[1], resource_path=q[2],
                                     intent=LockIntent(q[3]), acquired_at=when, is_active=True,
                                     saga_step_id=q[4] if len(q) > 4 else None)
                locks[lid] = lock
                ids = index.get(q[2])
                if ids is None:
                    index[q[2]] = [lid]
                else:
                    ids.append(lid)
                out[i] = lock
                continue
            err = self._refusal(q[0], q[2], LockIntent(q[3]))
            if err is not None:
                out[i] = err
                continue
            if ok[i] != 2:
                raise AssertionError("K20 refused a request the host check grants")
            # more readers than holder slots: granted here, the row is rebuilt
            out[i] = IntentLockManager.acquire(self, q[0], q[1], q[2], LockIntent(q[3]), q[4] if len(q) > 4 else None)
            self._dirty.add(q[2])
        return out

    def _refusal(self, agent: str, path: str, intent: LockIntent):
        """The error sequential :meth:`IntentLockManager.acquire` raises for a
        refused request (same message, same wait-for edges), or None when the
        records show no conflict.  Without wait-for edges no deadlock is possible
        (a conflict never involves the requester itself), so the search is skipped."""
        locks = self._locks
        read = intent is LockIntent.READ
        conflicts = [lk for lk in (locks[i] for i in self._resource_locks.get(path, ()) if i in locks)
                     if lk.is_active and lk.agent_did != agent and not (read and lk.intent == LockIntent.READ)]
        if not conflicts:
            return None
        blockers = {c.agent_did for c in conflicts}
        if self._wait_for and self._would_deadlock(agent, blockers):
            return DeadlockError(
                f"Deadlock detected: {agent} would wait on "
                f"{blockers} which are waiting on {agent}"
            )
        if self._record_waits:
            self._wait_for.setdefault(agent, set()).update(blockers)
        return LockContentionError(
            f"Lock contention on {path}: {agent} ({intent.value}) "
            f"conflicts with {', '.join(c.agent_did for c in conflicts)}"
        )

    def acquire_rows(self, agent_ids: torch.Tensor, resource_rows: torch.Tensor, intents: torch.Tensor) -> torch.Tensor:
        """Tensor-native K20: decide (and record in the device holder tables) a
        batch of acquires given as device tensors — int32 agent ids
        (:meth:`agent_row`) and resource rows (:meth:`resource_row`), u8 intents
        (0 read 1 write 2 exclusive) — → u8 per request on the device: 1
        granted, 0 refused (contention), 2 refused because the resource's 16
        holder slots belong to other agents.  No host lock records are made: the
        caller tracks its holds and returns them with :meth:`release_rows`."""
        self._sync()
        n = resource_rows.numel()
        rows = resource_rows.to(i32)
        sr, order = torch.sort(rows, stable=True)
        first = torch.ones(n, dtype=torch.bool, device=self.device)
        first[1:] = sr[1:] != sr[:-1]
        seg = torch.cat([torch.nonzero(first).flatten().to(i32), torch.tensor([n], dtype=i32, device=self.device)])
        granted = torch.empty(n, dtype=u8, device=self.device)
        SN.lock_grant(seg, order.to(i32), rows, agent_ids.to(i32), intents.to(u8), self._table, granted)
        return granted

    def release_rows(self, agent_ids: torch.Tensor, resource_rows: torch.Tensor, intents: torch.Tensor) -> torch.Tensor:
        """Return holds granted by :meth:`acquire_rows` (one lock of that intent
        per request) → u8 per request, 1 released, 0 not held."""
        return self.acquire_rows(agent_ids, resource_rows, intents.to(u8) | SN.LOCK_RELEASE)

    def resource_row(self, path: str) -> int:
        r = self._rid(path)
        self._sync()
        return r

    def agent_row(self, did: str) -> int:
        return self._aid(did)
