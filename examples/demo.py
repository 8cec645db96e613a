#!/usr/bin/env python3
"""Guided tour of the hypervisor (reference examples/demo.py covers the first
five topics; the sixth shows the MI355X batch engine).

    python examples/demo.py            # all demos
    python examples/demo.py saga audit # a subset

Demos: lifecycle, saga, liability, audit, integrations, engine.
"""

from __future__ import annotations

import asyncio
import os
import sys
from types import SimpleNamespace

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from hypervisor import ConsistencyMode, DeltaEngine, Hypervisor, HypervisorEventBus, SessionConfig  # noqa: E402
from hypervisor.audit.delta import VFSChange  # noqa: E402
from hypervisor.integrations.cmvk_adapter import CMVKAdapter  # noqa: E402
from hypervisor.integrations.iatp_adapter import IATPAdapter  # noqa: E402

USE_COLOR = sys.stdout.isatty()


def _c(code: str, s: str) -> str:
    return f"\033[{code}m{s}\033[0m" if USE_COLOR else s


def banner(title: str) -> None:
    print("\n" + _c("1;36", f"━━ {title} " + "━" * max(0, 70 - len(title))))


def say(msg: str) -> None:
    print("  " + _c("32", "›") + " " + msg)


async def demo_lifecycle() -> None:
    banner("1. Session lifecycle: create → join → activate → audit → terminate")
    bus = HypervisorEventBus()
    hv = Hypervisor(event_bus=bus)
    s = await hv.create_session(SessionConfig(enable_audit=True, consistency_mode=ConsistencyMode.EVENTUAL),
                                creator_did="did:mesh:admin")
    sid = s.sso.session_id
    say(f"session {sid} ({s.sso.state.value})")
    for did, sigma in [("did:mesh:lead", 0.97), ("did:mesh:worker", 0.72), ("did:mesh:intern", 0.31)]:
        ring = await hv.join_session(sid, did, sigma_raw=sigma)
        say(f"{did:20s} σ={sigma:.2f} → {ring.name}")
    await hv.activate_session(sid)
    s.sso.vfs.write("/workspace/plan.md", "# plan\n", "did:mesh:lead")
    s.delta_engine.capture("did:mesh:lead", [VFSChange("/workspace/plan.md", "add", "h-plan")])
    root = await hv.terminate_session(sid)
    say(f"terminated; Merkle root {root[:16]}…, committed={hv.commitment.verify(sid, root)}")
    say(f"events: {', '.join(e.event_type.value for e in bus.all_events)}")


async def demo_saga() -> None:
    banner("2. Saga: three steps, third fails, reverse-order compensation")
    hv = Hypervisor()
    s = await hv.create_session(SessionConfig(), "did:mesh:admin")
    saga = s.saga.create_saga(s.sso.session_id)
    names = ["provision-db", "migrate-schema", "deploy-api"]
    steps = [s.saga.add_step(saga.saga_id, n, "did:mesh:worker", f"/api/{n}",
                             undo_api=None if n == "migrate-schema" else f"/api/{n}/undo") for n in names]

    async def ok():
        return "done"

    async def boom():
        raise RuntimeError("deploy target unreachable")

    for st in steps:
        try:
            await s.saga.execute_step(saga.saga_id, st.step_id, boom if st.action_id == "deploy-api" else ok)
            say(f"{st.action_id:16s} {st.state.value}")
        except RuntimeError as e:
            say(f"{st.action_id:16s} {st.state.value}: {e}")
            break

    async def undo(step):
        return f"undid {step.action_id}"

    failed = await s.saga.compensate(saga.saga_id, undo)
    for st in steps:
        say(f"{st.action_id:16s} → {st.state.value}" + (f"  ({st.error})" if st.error else ""))
    say(f"saga {saga.state.value}; {len(failed)} compensation failure(s) reported as failures")


async def demo_liability() -> None:
    banner("3. Joint liability: vouch, bond, slash with cascade")
    hv = Hypervisor()
    s = await hv.create_session(SessionConfig(), "did:mesh:admin")
    sid = s.sso.session_id
    v1 = hv.vouching.vouch("did:mesh:senior", "did:mesh:mid", sid, 0.9)
    v2 = hv.vouching.vouch("did:mesh:mid", "did:mesh:new", sid, 0.7, bond_pct=0.5)
    say(f"senior→mid bond {v1.bonded_amount:.3f}; mid→new bond {v2.bonded_amount:.3f}")
    eff = hv.vouching.compute_sigma_eff("did:mesh:new", sid, 0.3, risk_weight=0.65)
    say(f"σ_eff(new) = min(0.30 + 0.65·{v2.bonded_amount:.2f}, 1) = {eff:.4f}")
    scores = {"did:mesh:senior": 0.9, "did:mesh:mid": 0.7, "did:mesh:new": 0.3}
    hv.slashing.slash("did:mesh:new", sid, 0.3, 0.95, "exfiltration attempt", scores)
    for r in hv.slashing.history:
        say(f"slash {r.vouchee_did} depth={r.cascade_depth}: " +
            ", ".join(f"{c.voucher_did} {c.sigma_before:.2f}→{c.sigma_after:.2f}" for c in r.voucher_clips))
    say(f"scores after: { {k: round(v, 3) for k, v in scores.items()} }")


async def demo_audit() -> None:
    banner("4. Audit: hash-chained deltas, Merkle root, tamper detection")
    de = DeltaEngine("session:demo")
    for i in range(5):
        de.capture("did:mesh:agent", [VFSChange(f"/f{i}", "add", f"h{i}")])
    say(f"{de.turn_count} deltas, root {de.compute_merkle_root()[:16]}…, chain ok={de.verify_chain()}")
    de._deltas[2].changes[0].path = "/etc/shadow"
    say(f"after tampering with delta 3: chain ok={de.verify_chain()} (verification does not self-repair)")


async def demo_integrations() -> None:
    banner("5. Integrations: IATP manifest onboarding, CMVK drift → slash")

    class Drift:
        def verify_embeddings(self, **kw):
            return SimpleNamespace(drift_score=0.82, explanation="goal divergence")

    hv = Hypervisor(iatp=IATPAdapter(), cmvk=CMVKAdapter(Drift()), demote_on_slash=True)
    s = await hv.create_session(SessionConfig(), "did:mesh:admin")
    sid = s.sso.session_id
    manifest = {"agent_id": "did:mesh:planner", "trust_level": "trusted", "trust_score": 8,
                "actions": [{"action_id": "write_doc", "reversibility": "full", "undo_api": "/undo"},
                            {"action_id": "send_email", "reversibility": "none"}]}
    ring = await hv.join_session(sid, "did:mesh:planner", manifest=manifest)
    say(f"manifest → σ hint 0.8 → {ring.name}; consistency forced to {s.sso.consistency_mode.value}")
    await hv.join_session(sid, "did:mesh:buddy", sigma_raw=0.9)
    hv.vouching.vouch("did:mesh:buddy", "did:mesh:planner", sid, 0.9)
    res = await hv.verify_behavior(sid, "did:mesh:planner", [1.0], [0.0])
    buddy = s.sso.get_participant("did:mesh:buddy")
    say(f"drift {res.drift_score:.2f} ({res.severity.value}) → slashed; voucher σ_eff {buddy.sigma_eff:.2f}, "
        f"ring {buddy.ring.name}")


async def demo_engine() -> None:
    banner("6. MI355X batched pipeline: the full pipeline for many sessions in one launch")
    import torch

    from hypervisor import Hypervisor

    dev = "cuda" if torch.cuda.is_available() else "cpu"
    n = 65536 if dev == "cuda" else 2048
    hv = Hypervisor(device=dev)
    hv.pipeline_batch(64)  # warm-up (agent registration, kernel load)
    import time

    t0 = time.perf_counter()
    run = hv.pipeline_batch(n)
    dt = time.perf_counter() - t0
    say(f"{n} sessions on {dev} in {dt * 1e3:.2f} ms ({run.ok} completed), written as ordinary store sessions")
    sid = run.session_ids[0]
    m = hv.get_session(sid)
    say(f"session {sid} root {run.roots[sid][:16]}… via the API: state={m.sso.state.value} "
        f"chain={m.delta_engine.verify_chain()} root-match={m.delta_engine.compute_merkle_root() == run.roots[sid]}")


DEMOS = {
    "lifecycle": demo_lifecycle,
    "saga": demo_saga,
    "liability": demo_liability,
    "audit": demo_audit,
    "integrations": demo_integrations,
    "engine": demo_engine,
}


def main(argv: list[str]) -> int:
    chosen = argv or list(DEMOS)
    for name in chosen:
        if name not in DEMOS:
            print(f"unknown demo {name!r}; choose from {', '.join(DEMOS)}")
            return 2
        asyncio.run(DEMOS[name]())
    print()
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
