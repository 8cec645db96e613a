"""§5.1 host-stage tracing: spans around the façade's lifecycle stages and the
saga orchestrator, per-stage summary and chrome-trace export."""

from __future__ import annotations

import json

from agent_hypervisor_amd.utils import tracing
from hypervisor import Hypervisor, SessionConfig


async def test_stage_spans_and_export(tmp_path):
    tracing.clear()
    tracing.set_tracing(True)
    try:
        hv = Hypervisor()
        for _ in range(3):
            m = await hv.create_session(SessionConfig(), "did:admin")
            sid = m.sso.session_id
            await hv.join_session(sid, "did:a", sigma_raw=0.8)
            await hv.activate_session(sid)
            g = m.saga.create_saga(sid)
            st = m.saga.add_step(g.saga_id, "a", "did:a", "/x")

            async def ok():
                return 1

            await m.saga.execute_step(g.saga_id, st.step_id, ok)
            await hv.terminate_session(sid)
        with tracing.span("custom", k=1):
            pass
    finally:
        tracing.set_tracing(False)
    s = tracing.summary()
    for name in ("hypervisor.create_session", "hypervisor.join_session", "hypervisor.activate_session",
                 "hypervisor.terminate_session", "saga.execute_step"):
        assert s[name]["count"] == 3 and s[name]["p50_us"] > 0
    path = tracing.export_chrome_trace(str(tmp_path / "t.json"))
    ev = json.load(open(path))["traceEvents"]
    assert any(e["name"] == "custom" and e["args"] == {"k": 1} for e in ev)


async def test_disabled_records_nothing():
    tracing.clear()
    hv = Hypervisor()
    await hv.create_session(SessionConfig(), "did:admin")
    assert tracing.spans() == []
