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


def _iso(t) -> Any:
    return t.isoformat() if t is not None else None


def summary(st, limit: int = 200) -> dict[str, Any]:
    """Every tab's data from the live hypervisor (capped at ``limit`` rows each)."""
    from hypervisor.core import LazyManagedSession

    hv, bus = st.hv, st.bus
    sessions = hv.sessions  # batched-pipeline sessions come as row proxies: nothing is built for the summary
    snaps = hv.snapshots(parts=True)  # one batched device read per segment, same order as hv.sessions
    rings: Counter = Counter()
    states: Counter = Counter()
    session_rows, agent_rows = [], []
    for m, x in zip(sessions, snaps):
        states[x.state.value] += 1
        for p in x.participants:
            rings[p.ring.name] += 1
            if len(agent_rows) < limit:
                agent_rows.append({"agent_did": p.agent_did, "session_id": x.session_id, "ring": int(p.ring),
                                   "ring_name": p.ring.name, "sigma_raw": round(p.sigma_raw, 4),
                                   "sigma_eff": round(p.sigma_eff, 4), "active": bool(p.is_active)})
        if len(session_rows) < limit:
            if isinstance(m, LazyManagedSession):
                turns = x.delta_count
            else:
                de = m.delta_engine
                turns = de.turn_count if de is not None else 0
            session_rows.append({"session_id": x.session_id, "state": x.state.value,
                                 "participants": x.participant_count, "created_at": _iso(x.created_at),
                                 "deltas": turns,
                                 "merkle_root": x.merkle_root if x.committed_at is not None else
                                 getattr(hv.commitment.get_commitment(x.session_id), "merkle_root", None)})
    sagas: Counter = Counter()
    steps: Counter = Counter()
    saga_rows = []
    for g in hv.saga_summaries():  # one column gather per field (batches from their rows)
        sagas[g["state"]] += 1
        for s_ in g["steps"]:
            steps[s_["state"]] += 1
        if len(saga_rows) < limit:
            saga_rows.append({
                "saga_id": g["saga_id"], "session_id": g["session_id"], "state": g["state"], "error": g["error"],
                "created_at": _iso(g["created_at"]), "completed_at": _iso(g["completed_at"]),
                "steps": [{"action_id": x["action_id"], "agent_did": x["agent_did"], "state": x["state"],
                           "retry_count": x["retry_count"], "error": x["error"], "started_at": _iso(x["started_at"]),
                           "completed_at": _iso(x["completed_at"])} for x in g["steps"]]})
    exposure: Counter = Counter()
    vouch_rows = []
    for v in hv.vouching.records():
        live = v.is_active and not v.is_expired
        if live:
            exposure[v.voucher_did] += v.bonded_amount
        if len(vouch_rows) < limit:
            vouch_rows.append({"voucher_did": v.voucher_did, "vouchee_did": v.vouchee_did, "session_id": v.session_id,
                               "bonded_amount": round(v.bonded_amount, 6), "pct": v.bonded_sigma_pct, "live": live})
    slash_rows = [{"vouchee_did": r.vouchee_did, "session_id": r.session_id, "reason": r.reason,
                   "depth": r.cascade_depth, "timestamp": _iso(r.timestamp),
                   "clips": [{"voucher_did": c.voucher_did, "before": round(c.sigma_before, 4),
                              "after": round(c.sigma_after, 4)} for c in r.voucher_clips]}
                  for r in list(hv.slashing.history)[-limit:]]
    ring_events = [e.to_dict() for e in bus.query(limit=limit) if e.event_type.value.startswith("ring.")][::-1]
    events = [e.to_dict() for e in bus.query(limit=limit)][::-1]
    engine = None
    if getattr(hv, "batched_sessions", 0):  # sessions written by batched device launches (store rows)
        engine = {"device": str(hv._store.device), "batched_sessions": hv.batched_sessions,
                  "live_rows": hv._store.live_rows()}
    store = getattr(hv, "_store", None)
    return {
        "overview": {
            "sessions": len(sessions),
            "active_sessions": sum(1 for x in snaps if x.state.value not in ("archived", "terminating")),
            "participants": sum(x.participant_count for x in snaps),
            "vouches": len(hv.vouching.records()),
            "slashes": len(hv.slashing.history),
            "commitments": hv.commitment.commitment_count,
            "events": bus.event_count,
            "session_states": dict(states),
            "state_authority": "device" if store is not None else "host",
        },
        "sessions": session_rows,
        "rings": dict(rings),
        "agents": agent_rows,
        "ring_events": ring_events,
        "sagas": {"by_state": dict(sagas), "steps_by_state": dict(steps), "rows": saga_rows},
        "liability": {"top_exposure": [{"agent_did": a, "exposure": round(x, 6)} for a, x in exposure.most_common(10)],
                      "vouches": vouch_rows, "slashes": slash_rows},
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
 td,th{border-bottom:1px solid #2a2f3a;padding:5px 8px;text-align:left;vertical-align:top} th{color:#9aa4b2;font-weight:500}
 .bar{background:#4c8dff;height:10px} .muted{color:#9aa4b2} .row{display:flex;gap:24px;flex-wrap:wrap}
 .row>div{flex:1;min-width:380px} input{background:#161a22;color:#e6e6e6;border:1px solid #2a2f3a;padding:4px 8px}
 .st-committed,.st-completed,.st-active{color:#5cd68a} .st-failed,.st-escalated,.st-compensation_failed{color:#ff6b6b}
 .st-compensated,.st-compensating{color:#f5c451} code{font-size:12px;color:#9aa4b2}
</style></head><body>
<header><h1>Agent Hypervisor <span class="muted">— live state, refreshed every 2 s</span></h1>
<nav id="tabs"></nav></header><main id="main">loading…</main>
<script>
const TABS=["Overview","Rings","Sagas","Liability","Events"];let tab="Overview",data=null,filt="";
const RC=["#ff6b6b","#f5c451","#4c8dff","#5cd68a"];
function esc(x){return String(x??"").replace(/[&<>]/g,c=>({"&":"&amp;","<":"&lt;",">":"&gt;"}[c]))}
function nav(){document.getElementById("tabs").innerHTML=TABS.map(t=>
 `<button class="${t==tab?"on":""}" onclick="tab='${t}';render()">${t}</button>`).join("")}
function kv(o){return Object.entries(o||{}).map(([k,v])=>`<tr><td>${esc(k)}</td><td>${esc(v)}</td></tr>`).join("")}
function bars(o){const m=Math.max(1,...Object.values(o||{}));return Object.entries(o||{}).map(([k,v])=>
 `<tr><td>${esc(k)}</td><td>${v}</td><td style="width:60%"><div class="bar" style="width:${100*v/m}%"></div></td></tr>`).join("")}
function table(rows,cols){return `<table><tr>${cols.map(c=>`<th>${c}</th>`).join("")}</tr>`+rows.map(r=>
 `<tr>${cols.map(c=>`<td class="${c=="state"?"st-"+r[c]:""}">${esc(typeof r[c]=="object"&&r[c]!==null?JSON.stringify(r[c]):r[c])}</td>`).join("")}</tr>`).join("")+`</table>`}
function scatter(agents){  // σ_eff vs ring (SVG)
 const W=520,H=200;let s=`<svg width="${W}" height="${H}" style="background:#161a22;border-radius:8px">`;
 for(let r=0;r<4;r++)s+=`<text x="4" y="${30+r*45}" fill="#9aa4b2" font-size="11">R${r}</text>`;
 agents.forEach(a=>{const x=40+a.sigma_eff*(W-60),y=26+a.ring*45+(Math.random()*8-4);
  s+=`<circle cx="${x}" cy="${y}" r="4" fill="${RC[a.ring]}"><title>${esc(a.agent_did)} σ_eff=${a.sigma_eff}</title></circle>`});
 return s+`<text x="${W-70}" y="${H-6}" fill="#9aa4b2" font-size="11">σ_eff →</text></svg>`}
function gantt(rows){  // step timelines per saga (SVG)
 const steps=rows.flatMap(g=>g.steps.filter(s=>s.started_at).map(s=>({g:g.saga_id,...s})));if(!steps.length)return"";
 const t=x=>Date.parse(x);const t0=Math.min(...steps.map(s=>t(s.started_at))),t1=Math.max(...steps.map(s=>t(s.completed_at||s.started_at)))+1;
 const W=760,rh=14;let s=`<svg width="${W}" height="${rows.length*rh+20}" style="background:#161a22;border-radius:8px">`;
 rows.forEach((g,i)=>g.steps.forEach(st=>{if(!st.started_at)return;const a=t(st.started_at),b=t(st.completed_at||st.started_at)+1;
  const col={committed:"#5cd68a",compensated:"#f5c451",failed:"#ff6b6b",compensation_failed:"#ff6b6b"}[st.state]||"#4c8dff";
  s+=`<rect x="${150+(a-t0)/(t1-t0)*(W-160)}" y="${4+i*rh}" width="${Math.max(2,(b-a)/(t1-t0)*(W-160))}" height="${rh-4}" fill="${col}"><title>${esc(st.action_id)} ${st.state}</title></rect>`}));
 rows.forEach((g,i)=>s+=`<text x="4" y="${14+i*rh}" fill="#9aa4b2" font-size="10">${esc(g.saga_id.slice(0,22))}</text>`);
 return s+"</svg>"}
function render(){nav();if(!data)return;const d=data,m=document.getElementById("main");
 if(tab=="Overview"){const o=d.overview;m.innerHTML=`<div class="cards">${["sessions","active_sessions",
  "participants","vouches","slashes","commitments","events","state_authority"].map(k=>`<div class="card">${k}<b>${o[k]}</b></div>`).join("")}
  </div><div class="row"><div><h3>Session states</h3><table>${bars(o.session_states)}</table></div>`+
  (d.engine?`<div><h3>Batched device engine</h3><table>${kv(d.engine)}</table></div>`:"")+`</div>`+
  `<h3>Sessions</h3>`+table(d.sessions,["session_id","state","participants","deltas","created_at","merkle_root"])}
 if(tab=="Rings")m.innerHTML=`<div class="row"><div><h3>Participants per ring</h3><table>${bars(d.rings)}</table></div>
  <div><h3>σ_eff vs ring</h3>${scatter(d.agents)}</div></div><h3>Ring transitions</h3>`+
  table(d.ring_events,["timestamp","event_type","agent_did","session_id","payload"])+`<h3>Agents</h3>`+
  table(d.agents,["agent_did","session_id","ring_name","sigma_raw","sigma_eff","active"]);
 if(tab=="Sagas")m.innerHTML=`<div class="row"><div><h3>Sagas</h3><table>${bars(d.sagas.by_state)}</table></div>
  <div><h3>Steps</h3><table>${bars(d.sagas.steps_by_state)}</table></div></div><h3>Timeline</h3>${gantt(d.sagas.rows.slice(-30))}
  <h3>Sagas and compensation chains</h3><table><tr><th>saga</th><th>state</th><th>steps (in order)</th><th>error</th></tr>`+
  d.sagas.rows.map(g=>`<tr><td><code>${esc(g.saga_id)}</code></td><td class="st-${g.state}">${g.state}</td><td>`+
  g.steps.map(s=>`<span class="st-${s.state}">${esc(s.action_id)}:${s.state}${s.retry_count?` (retry ${s.retry_count})`:""}</span>`).join(" → ")+
  `</td><td class="muted">${esc(g.error||"")}</td></tr>`).join("")+`</table>`;
 if(tab=="Liability")m.innerHTML=`<div class="row"><div><h3>Top exposure (Σ live bonds)</h3><table>`+
  d.liability.top_exposure.map(r=>`<tr><td>${esc(r.agent_did)}</td><td>${r.exposure}</td></tr>`).join("")+`</table></div>
  <div><h3>Slash history (cascades)</h3><table><tr><th>vouchee</th><th>depth</th><th>reason</th><th>clipped vouchers</th></tr>`+
  d.liability.slashes.map(s=>`<tr><td>${esc(s.vouchee_did)}</td><td>${s.depth}</td><td>${esc(s.reason)}</td><td>`+
  s.clips.map(c=>`${esc(c.voucher_did)} ${c.before}→${c.after}`).join("<br>")+`</td></tr>`).join("")+`</table></div></div>
  <h3>Vouch edges</h3>`+table(d.liability.vouches,["voucher_did","vouchee_did","session_id","bonded_amount","pct","live"]);
 if(tab=="Events"){const ev=d.events.recent.filter(e=>!filt||JSON.stringify(e).includes(filt));
  m.innerHTML=`<div class="row"><div><h3>By type</h3><table>${bars(d.events.by_type)}</table></div></div>
  <h3>Stream <input placeholder="filter" value="${esc(filt)}" oninput="filt=this.value;render()"></h3>`+
  table(ev,["timestamp","event_type","session_id","agent_did","payload"])}}
async function poll(){try{data=await (await fetch("/api/v1/dashboard/summary")).json();render()}catch(e){}
 setTimeout(poll,2000)}
nav();poll();
</script></body></html>
"""


@router.get("/dashboard", response_class=HTMLResponse, tags=["Dashboard"])
async def dashboard_page() -> str:
    return _PAGE
