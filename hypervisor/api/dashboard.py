"""Live dashboard (reference examples/dashboard/app.py, C49).

The reference's Streamlit dashboard renders *synthetic* data even when the
hypervisor is importable.  This one is a self-contained HTML page served by the
REST app at ``/dashboard``; it polls ``/api/v1/dashboard/summary``, which
aggregates the live state of the serving :class:`Hypervisor` (and of its
device engine when one exists): overview counters, ring distribution, saga
states, top liability exposures and recent events — the same five tabs.
"""

from __future__ import annotations

from collections import Counter
from typing import Any

from fastapi import APIRouter, Request
from fastapi.responses import HTMLResponse

router = APIRouter()


def summary(st) -> dict[str, Any]:
    hv, bus = st.hv, st.bus
    sessions = hv.sessions
    rings: Counter = Counter()
    states: Counter = Counter()
    for m in sessions:
        states[m.sso.state.value] += 1
        for p in m.sso.participants:
            rings[p.ring.name] += 1
    sagas: Counter = Counter()
    steps: Counter = Counter()
    for m in sessions:
        for g in m.saga.sagas:
            sagas[g.state.value] += 1
            for s in g.steps:
                steps[s.state.value] += 1
    exposure: Counter = Counter()
    for v in hv.vouching.records():
        if v.is_active and not v.is_expired:
            exposure[v.voucher_did] += v.bonded_amount
    events = [e.to_dict() for e in bus.query(limit=25)][::-1]
    engine = None
    if hv._device_engine is not None:
        eng = hv._device_engine
        t = eng.sessions
        engine = {
            "device": str(eng.device),
            "session_capacity": t.capacity,
            "agents": eng.agents.count,
            "archived_rows": int((t.sess_state == 4).sum().item()),
            "table_bytes": t.nbytes() if hasattr(t, "nbytes") else None,
        }
    return {
        "overview": {
            "sessions": len(sessions),
            "active_sessions": len(hv.active_sessions),
            "participants": sum(m.sso.participant_count for m in sessions),
            "vouches": len(hv.vouching.records()),
            "slashes": len(hv.slashing.history),
            "commitments": hv.commitment.commitment_count,
            "events": bus.event_count,
            "session_states": dict(states),
        },
        "rings": dict(rings),
        "sagas": {"by_state": dict(sagas), "steps_by_state": dict(steps)},
        "liability": {"top_exposure": [{"agent_did": a, "exposure": round(x, 6)} for a, x in exposure.most_common(10)]},
        "events": {"by_type": bus.type_counts(), "recent": events},
        "engine": engine,
    }


@router.get("/api/v1/dashboard/summary", tags=["Dashboard"])
async def dashboard_summary(request: Request) -> dict[str, Any]:
    from hypervisor.api.server import _state

    return summary(_state(request))


_PAGE = """<!doctype html>
<html lang="en"><head><meta charset="utf-8"><title>Agent Hypervisor — live</title>
<style>
 body{font:14px system-ui,sans-serif;margin:0;background:#0f1115;color:#e6e6e6}
 header{padding:12px 20px;background:#161a22;border-bottom:1px solid #2a2f3a}
 h1{font-size:18px;margin:0} nav button{background:none;border:0;color:#9aa4b2;padding:8px 12px;cursor:pointer}
 nav button.on{color:#fff;border-bottom:2px solid #4c8dff} main{padding:16px 20px}
 .cards{display:flex;gap:12px;flex-wrap:wrap} .card{background:#161a22;border:1px solid #2a2f3a;border-radius:8px;
 padding:12px 16px;min-width:140px} .card b{display:block;font-size:22px} table{border-collapse:collapse;width:100%}
 td,th{border-bottom:1px solid #2a2f3a;padding:6px 8px;text-align:left} .bar{background:#4c8dff;height:10px}
 .muted{color:#9aa4b2}
</style></head><body>
<header><h1>Agent Hypervisor <span class="muted">— live state, refreshed every 2 s</span></h1>
<nav id="tabs"></nav></header><main id="main">loading…</main>
<script>
const TABS=["Overview","Rings","Sagas","Liability","Events"];let tab="Overview",data=null;
function nav(){document.getElementById("tabs").innerHTML=TABS.map(t=>
 `<button class="${t==tab?"on":""}" onclick="tab='${t}';render()">${t}</button>`).join("")}
function kv(o){return Object.entries(o||{}).map(([k,v])=>`<tr><td>${k}</td><td>${v}</td></tr>`).join("")}
function bars(o){const m=Math.max(1,...Object.values(o||{}));return Object.entries(o||{}).map(([k,v])=>
 `<tr><td>${k}</td><td>${v}</td><td style="width:60%"><div class="bar" style="width:${100*v/m}%"></div></td></tr>`).join("")}
function render(){nav();if(!data)return;const d=data,m=document.getElementById("main");
 if(tab=="Overview"){const o=d.overview;m.innerHTML=`<div class="cards">${["sessions","active_sessions",
  "participants","vouches","slashes","commitments","events"].map(k=>`<div class="card">${k}<b>${o[k]}</b></div>`).join("")}
  </div><h3>Session states</h3><table>${bars(o.session_states)}</table>`+(d.engine?`<h3>Device engine</h3><table>${kv(d.engine)}</table>`:"")}
 if(tab=="Rings")m.innerHTML=`<h3>Participants per ring</h3><table>${bars(d.rings)}</table>`;
 if(tab=="Sagas")m.innerHTML=`<h3>Sagas</h3><table>${bars(d.sagas.by_state)}</table><h3>Steps</h3><table>${bars(d.sagas.steps_by_state)}</table>`;
 if(tab=="Liability")m.innerHTML=`<h3>Top exposure (Σ active bonds)</h3><table>`+
  d.liability.top_exposure.map(r=>`<tr><td>${r.agent_did}</td><td>${r.exposure}</td></tr>`).join("")+`</table>`;
 if(tab=="Events")m.innerHTML=`<h3>By type</h3><table>${bars(d.events.by_type)}</table><h3>Recent</h3><table>`+
  d.events.recent.map(e=>`<tr><td class="muted">${e.timestamp}</td><td>${e.event_type}</td><td>${e.session_id||""}</td><td>${e.agent_did||""}</td></tr>`).join("")+`</table>`;}
async function poll(){try{data=await (await fetch("/api/v1/dashboard/summary")).json();render()}catch(e){}
 setTimeout(poll,2000)}
nav();poll();
</script></body></html>
"""


@router.get("/dashboard", response_class=HTMLResponse, tags=["Dashboard"])
async def dashboard_page() -> str:
    return _PAGE
