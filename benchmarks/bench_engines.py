"""Throughput of the stand-alone governance engines: host Python engine (the
reference's per-call loop) vs the device-resident variant's batched kernel path.

For each engine one workload of ``--calls`` operations is replayed (pinned clock
so host and device see the same instants) and timed three ways where they exist:

* ``host``   — the host engine, one Python call per operation;
* ``batch``  — the device engine's tuple batch API (Python grouping + one launch);
* ``tensor`` — the device engine's tensor API (inputs already on the device, the
  grouping is a device sort; output left on the device).

Every workload is ``--calls`` operations (100 k by default; the host loops are
timed on the first ``--host-calls`` of them).

Prints one JSON line per (engine, path) with ops/s and µs per batch.  Kernels:
K16 breach, K17 bucket, K18 expiry, K22 ledger + drift, K19 vector clocks, K20
lock contention, K02 ring check, K21 attribution.
"""

from __future__ import annotations

import argparse
import json
import os
import random
import sys
import time
from datetime import datetime, timedelta, timezone

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from agent_hypervisor_amd.ops import ledger as LG  # noqa: E402
from agent_hypervisor_amd.ops import rings as RG  # noqa: E402

from hypervisor import _clock  # noqa: E402
from hypervisor.integrations.cmvk_adapter import CMVKAdapter  # noqa: E402
from hypervisor.liability.attribution import CausalAttributor  # noqa: E402
from hypervisor.liability.ledger import LedgerEntryType, LiabilityLedger  # noqa: E402
from hypervisor.liability.quarantine import QuarantineManager, QuarantineReason  # noqa: E402
from hypervisor.models import ActionDescriptor, ExecutionRing, ReversibilityLevel  # noqa: E402
from hypervisor.rings.breach_detector import RingBreachDetector  # noqa: E402
from hypervisor.rings.enforcer import RingEnforcer  # noqa: E402
from hypervisor.security.rate_limiter import AgentRateLimiter  # noqa: E402
from hypervisor.session.intent_locks import IntentLockManager, LockIntent  # noqa: E402
from hypervisor.session.vector_clock import VectorClockManager  # noqa: E402

R = list(ExecutionRing)
T0 = datetime(2026, 3, 1, tzinfo=timezone.utc)


def sync(dev):
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)


def timed(fn, dev, reps: int = 3) -> float:
    fn()  # warm (allocations, first launch)
    sync(dev)
    best = float("inf")
    for _ in range(reps):
        t = time.perf_counter()
        fn()
        sync(dev)
        best = min(best, time.perf_counter() - t)
    return best


def emit(engine: str, path: str, ops: int, sec: float, **extra) -> None:
    print(json.dumps(dict(engine=engine, path=path, ops=ops, ops_per_s=round(ops / sec, 1),
                          us_per_batch=round(sec * 1e6, 1), **extra)), flush=True)


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--calls", type=int, default=100_000)
    ap.add_argument("--profiles", type=int, default=10_000)
    ap.add_argument("--host-calls", type=int, default=20_000, help="host loops are timed on this many ops")
    ap.add_argument("--device", default="cuda" if torch.cuda.is_available() else "cpu")
    a = ap.parse_args()
    dev = torch.device(a.device)
    rng = random.Random(0)
    clk = [T0]
    _clock.set_clock(lambda: clk[0])
    n, P, nh = a.calls, a.profiles, a.host_calls

    # ---------------- K16 breach
    keys = [(f"did:a{i}", f"s{i % 7}") for i in range(P)]
    pick = [rng.randrange(P) for _ in range(n)]
    ar = [R[1 + (i % 3)] for i in pick]
    cr = [rng.choice(R) for _ in pick]
    calls = [(keys[i][0], keys[i][1], x, y) for i, x, y in zip(pick, ar, cr)]
    host = RingBreachDetector()
    emit("breach", "host", nh, timed(lambda: [host.record_call(*c) for c in calls[:nh]], torch.device("cpu"), 1))
    d = RingBreachDetector(device=dev, capacity=P)
    emit("breach", "batch", n, timed(lambda: d.record_calls_batch(calls), dev))
    rows = d.rows_for(keys)
    idx = torch.tensor(pick, device=dev)
    brow, bar = rows[idx], torch.tensor([x.value for x in ar], dtype=torch.uint8, device=dev)
    bcr = torch.tensor([y.value for y in cr], dtype=torch.uint8, device=dev)
    emit("breach", "tensor", n, timed(lambda: d.record_rows(brow, bar, bcr), dev), events=d.breach_count)

    # ---------------- K17 buckets
    reqs = [(keys[i][0], keys[i][1], R[i % 4], 1.0) for i in pick]
    hl = AgentRateLimiter()
    emit("rate_limit", "host", nh, timed(lambda: [hl.try_check(*q) for q in reqs[:nh]], torch.device("cpu"), 1))
    dl = AgentRateLimiter(device=dev, capacity=P)
    emit("rate_limit", "batch", n, timed(lambda: dl.check_batch(reqs), dev))
    lrows = dl.rows_for([(k[0], k[1], R[i % 4]) for i, k in enumerate(keys)])[idx]
    emit("rate_limit", "tensor", n, timed(lambda: dl.check_rows(lrows), dev))

    # ---------------- K18 expiry tick (quarantine)
    hq, dq = QuarantineManager(), QuarantineManager(device=dev, capacity=n)
    qs = [(f"did:q{i}", "s", QuarantineReason.MANUAL, "", rng.choice([60, 600, 3600])) for i in range(n)]
    hq.quarantine_batch(qs[:nh])
    dq.quarantine_batch(qs)
    clk[0] = T0 + timedelta(seconds=300)
    emit("quarantine_tick", "host", nh, timed(lambda: hq.tick(), torch.device("cpu"), 1))
    emit("quarantine_tick", "batch", n, timed(lambda: dq.tick(), dev))

    # ---------------- K22 ledger
    types = list(LedgerEntryType)
    hlg, dlg = LiabilityLedger(), LiabilityLedger(device=dev, capacity=n)
    agents = [f"did:l{i}" for i in range(P)]
    for k in range(n):
        e = (agents[rng.randrange(P)], rng.choice(types), "s", rng.random())
        dlg.record(*e)
        if k < nh:
            hlg.record(*e)
    emit("ledger_risk", "host", P, timed(lambda: hlg.compute_risk_profiles(agents), torch.device("cpu"), 1),
         entries=nh)
    emit("ledger_risk", "batch", P, timed(lambda: dlg.compute_risk_profiles(agents), dev), entries=n)

    # ---------------- K19 vector clocks
    va = [f"did:v{i}" for i in range(64)]
    vp = [f"/p{i}" for i in range(1024)]
    vops = [(rng.choice(["read", "write"]), rng.choice(vp), rng.choice(va)) for _ in range(n)]
    emit("vector_clock", "host", nh,
         timed(lambda: VectorClockManager().apply_batch(vops[:nh]), torch.device("cpu"), 1))
    emit("vector_clock", "batch", len(vops), timed(lambda: VectorClockManager(device=dev).apply_batch(vops), dev))

    # ---------------- K20 locks
    lreq = [(f"did:k{rng.randrange(256)}", "s", f"/r{rng.randrange(4096)}", rng.choice(list(LockIntent)))
            for _ in range(n)]
    emit("intent_locks", "host", len(lreq), timed(lambda: IntentLockManager().acquire_batch(lreq),
                                                  torch.device("cpu"), 1))
    emit("intent_locks", "batch", len(lreq), timed(lambda: IntentLockManager(device=dev).acquire_batch(lreq), dev))
    lm = IntentLockManager(device=dev)
    l_ag = torch.tensor([lm.agent_row(q[0]) for q in lreq], dtype=torch.int32, device=dev)
    l_rs = torch.tensor([lm.resource_row(q[2]) for q in lreq], dtype=torch.int32, device=dev)
    l_it = torch.tensor([{"read": 0, "write": 1, "exclusive": 2}[q[3].value] for q in lreq], dtype=torch.uint8,
                        device=dev)

    def rows_cycle():  # acquire the batch, then release what was granted
        g = lm.acquire_rows(l_ag, l_rs, l_it)
        k = g == 1
        lm.release_rows(l_ag[k], l_rs[k], l_it[k])
    emit("intent_locks", "tensor", len(lreq), timed(rows_cycle, dev), note="acquire_rows + release_rows")

    # ---------------- K02 ring check
    enf = RingEnforcer()
    revs = list(ReversibilityLevel)
    acts = [ActionDescriptor(action_id=f"a{i}", name="x", execute_api="/x", is_admin=i % 11 == 0,
                             is_read_only=i % 3 == 0, reversibility=revs[i % len(revs)]) for i in range(n)]
    rings = [R[i % 4] for i in range(n)]
    sig = [rng.random() for _ in range(n)]
    emit("ring_check", "host", nh, timed(lambda: [enf.check(r, x, s) for r, x, s in zip(rings[:nh], acts, sig)],
                                         torch.device("cpu"), 1))
    emit("ring_check", "batch", n, timed(lambda: enf.check_batch(rings, acts, sig, device=dev), dev),
         note="decisions as arrays; RingCheckResult objects built on access")
    emit("ring_check", "batch_materialized", n, timed(lambda: list(enf.check_batch(rings, acts, sig, device=dev)),
                                                      dev), note="every RingCheckResult built")
    u8 = torch.uint8
    t_ring = torch.tensor([r.value for r in rings], dtype=u8, device=dev)
    t_flag = torch.tensor([RG.action_flags(x.is_admin, x.is_read_only, x.required_ring is R[1]) for x in acts],
                          dtype=u8, device=dev)
    t_sig = torch.tensor(sig, dtype=torch.float64, device=dev)
    t_zero = torch.zeros(n, dtype=u8, device=dev)
    emit("ring_check", "tensor", n, timed(lambda: RG.ring_check(t_ring, t_flag, t_sig, t_zero, t_zero), dev))

    # ---------------- K21 attribution
    cases = []
    for c in range(n):
        ag = [f"did:x{j}" for j in range(rng.randint(2, 8))]
        acts_c = {x: [{"action_id": f"act{rng.randint(0, 5)}", "step_id": f"st{rng.randint(0, 4)}",
                       "success": rng.random() < 0.6} for _ in range(rng.randint(1, 5))] for x in ag}
        cases.append(dict(saga_id=f"saga{c}", session_id="s", agent_actions=acts_c, failure_step_id="st0",
                          failure_agent_did=ag[0]))
    emit("attribution", "host", nh, timed(lambda: [CausalAttributor().attribute(**c) for c in cases[:nh]],
                                          torch.device("cpu"), 1))
    emit("attribution", "batch", len(cases), timed(lambda: CausalAttributor().attribute_batch(cases, device=dev), dev))
    # tensor-native: the same cases as CSR columns already on the device
    no, ao, aof, sc_, rc_, om_ = [0], [0], [], [], [], []
    for c in cases:
        ags = list(c["agent_actions"])
        for j, a_ in enumerate(ags):
            for x in c["agent_actions"][a_]:
                aof.append(j)
                sc_.append(1 if x["success"] else 0)
                rc_.append(1 if (x["step_id"] == c["failure_step_id"] and a_ == c["failure_agent_did"]) else 0)
                om_.append(0.5)
        no.append(len(aof))
        ao.append(ao[-1] + len(ags))
    ti = lambda v, dt=torch.int32: torch.tensor(v, dtype=dt, device=dev)  # noqa: E731
    t_args = (ti(no), ti(ao), ti(aof), ti(sc_, torch.uint8), ti(rc_, torch.uint8), ti(om_, torch.float64))
    emit("attribution", "tensor", len(cases), timed(lambda: CausalAttributor().attribute_tensors(*t_args), dev))

    # ---------------- K22 drift
    drift = torch.rand(n, dtype=torch.float64, device=dev)
    dids = [f"did:d{i % 97}" for i in range(n)]
    emit("drift", "tensor", n, timed(lambda: LG.drift_severity(drift), dev))
    emit("drift", "batch", n, timed(lambda: CMVKAdapter().record_drift_batch(dids, ["s"] * n, drift, device=dev), dev))


if __name__ == "__main__":
    main()
