"""The guided demo runs end to end on the CPU host twins (reference C48)."""

from __future__ import annotations

import importlib.util
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_demo_runs_all_sections(capsys):
    spec = importlib.util.spec_from_file_location("ahv_demo", os.path.join(ROOT, "examples", "demo.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    assert mod.main([]) == 0
    out = capsys.readouterr().out
    for needle in ("Session lifecycle", "compensation_failed", "depth=1", "chain ok=False", "critical",
                   "root-match=True"):
        assert needle in out
    assert mod.main(["bogus"]) == 2


def test_dashboard_example_workload_feeds_every_tab():
    import asyncio
    import importlib.util
    import os
    import random

    from hypervisor import Hypervisor
    from hypervisor.api.dashboard import summary
    from hypervisor.api.server import ApiState
    from hypervisor.observability.event_bus import HypervisorEventBus

    path = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "examples", "dashboard", "app.py")
    spec = importlib.util.spec_from_file_location("dashboard_app", path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    bus = HypervisorEventBus()
    hv = Hypervisor(event_bus=bus)

    async def go():
        rnd = random.Random(7)
        for k in range(8):
            await mod.workload_round(hv, rnd, k)

    asyncio.run(go())
    s = summary(ApiState(bus=bus, hv=hv))
    o = s["overview"]
    assert o["sessions"] == 8 and o["vouches"] > 0 and o["slashes"] > 0 and o["commitments"] == 4
    assert len(s["rings"]) >= 2 and "escalated" in s["sagas"]["by_state"]
    assert s["events"]["recent"]


def test_batch_pipelines_example(capsys, monkeypatch):
    import asyncio

    import torch

    monkeypatch.setattr(torch.cuda, "is_available", lambda: False)  # the CPU twin here
    spec = importlib.util.spec_from_file_location("ahv_batch_example",
                                                  os.path.join(ROOT, "examples", "batch_pipelines.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    asyncio.run(mod.main())
    out = capsys.readouterr().out
    assert "template: 20000 sessions ok" in out and "verify_audit: ok=True" in out
