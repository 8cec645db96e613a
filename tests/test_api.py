"""REST front-end: every route of the reference server (reference
api/server.py:138-645) through FastAPI's TestClient, plus the batch-engine
extension on the CPU host twin."""

from __future__ import annotations

import pytest
from fastapi.testclient import TestClient

from hypervisor.api import create_app


@pytest.fixture()
def client():
    with TestClient(create_app()) as c:
        yield c


def _session(client, **kw) -> str:
    r = client.post("/api/v1/sessions", json={"creator_did": "did:mesh:admin", **kw})
    assert r.status_code == 201, r.text
    body = r.json()
    assert body["state"] == "handshaking" and body["consistency_mode"] == kw.get("consistency_mode", "eventual")
    return body["session_id"]


def test_health_and_stats(client):
    r = client.get("/health")
    assert r.status_code == 200 and r.json()["status"] == "ok"
    s = client.get("/api/v1/stats").json()
    assert s["total_sessions"] == 0 and s["event_count"] == 0 and s["version"]


def test_route_count_matches_reference(client):
    paths = client.get("/openapi.json").json()["paths"]
    routes = {(m.upper(), p) for p, ops in paths.items() for m in ops}
    routes -= {("POST", "/api/v1/engine/pipeline"), ("GET", "/dashboard"), ("GET", "/api/v1/dashboard/summary"),
               ("GET", "/api/v1/audit/verify")}  # extensions beyond the reference
    assert len(routes) == 21


def test_session_lifecycle_over_http(client):
    sid = _session(client)
    r = client.post(f"/api/v1/sessions/{sid}/join", json={"agent_did": "did:a", "sigma_raw": 0.8})
    assert r.status_code == 200
    assert r.json() == {"agent_did": "did:a", "session_id": sid, "assigned_ring": 2, "ring_name": "RING_2_STANDARD"}
    client.post(f"/api/v1/sessions/{sid}/join", json={"agent_did": "did:b", "sigma_raw": 0.3})
    # below min_sigma_eff → 400 (not a ValueError)
    assert client.post(f"/api/v1/sessions/{sid}/join", json={"agent_did": "did:c", "sigma_raw": 0.1}).status_code in (
        200, 400)
    assert client.post(f"/api/v1/sessions/{sid}/activate").json() == {"session_id": sid, "state": "active"}
    det = client.get(f"/api/v1/sessions/{sid}").json()
    assert det["state"] == "active" and det["participant_count"] >= 2
    assert {p["agent_did"] for p in det["participants"]} >= {"did:a", "did:b"}
    rings = client.get(f"/api/v1/sessions/{sid}/rings").json()
    assert "did:a" in rings["distribution"]["RING_2_STANDARD"]
    ar = client.get("/api/v1/agents/did:a/ring").json()
    assert ar["ring"] == 2 and ar["session_id"] == sid
    assert client.get("/api/v1/agents/did:nobody/ring").status_code == 404
    listed = client.get("/api/v1/sessions", params={"state": "active"}).json()
    assert [x["session_id"] for x in listed] == [sid]
    t = client.post(f"/api/v1/sessions/{sid}/terminate").json()
    assert t["state"] == "archived" and "merkle_root" in t
    assert client.get("/api/v1/sessions", params={"state": "active"}).json() == []
    s = client.get("/api/v1/stats").json()
    assert s["total_sessions"] == 1 and s["active_sessions"] == 0


def test_not_found_mapping(client):
    assert client.get("/api/v1/sessions/nope").status_code == 404
    assert client.post("/api/v1/sessions/nope/join", json={"agent_did": "x"}).status_code == 404
    assert client.post("/api/v1/sessions/nope/activate").status_code == 404
    assert client.post("/api/v1/sessions/nope/terminate").status_code == 404
    assert client.get("/api/v1/sagas/nope").status_code == 404
    assert client.post("/api/v1/sagas/nope/steps", json={"action_id": "a", "agent_did": "d",
                                                          "execute_api": "/x"}).status_code == 404
    assert client.get("/api/v1/sessions/nope/vouches").status_code == 404


def test_ring_check(client):
    action = {"action_id": "rm", "name": "rm", "execute_api": "/rm", "reversibility": "none"}
    r = client.post("/api/v1/rings/check", json={"agent_ring": 2, "action": action, "sigma_eff": 0.99})
    body = r.json()
    assert r.status_code == 200 and body["required_ring"] == 1 and not body["allowed"]
    assert body["requires_consensus"]
    read = {"action_id": "r", "name": "r", "execute_api": "/r", "is_read_only": True}
    body = client.post("/api/v1/rings/check", json={"agent_ring": 3, "action": read, "sigma_eff": 0.1}).json()
    assert body["allowed"] and body["reason"] == "Access granted"


def test_saga_routes(client):
    sid = _session(client)
    saga = client.post(f"/api/v1/sessions/{sid}/sagas").json()
    gid = saga["saga_id"]
    assert saga["state"] == "running"
    st = client.post(f"/api/v1/sagas/{gid}/steps", json={"action_id": "deploy", "agent_did": "did:a",
                                                         "execute_api": "/deploy", "undo_api": "/undo"})
    assert st.status_code == 201 and st.json()["state"] == "pending"
    step_id = st.json()["step_id"]
    ex = client.post(f"/api/v1/sagas/{gid}/steps/{step_id}/execute").json()
    assert ex["state"] == "committed" and ex["error"] is None
    # executing again is an invalid transition → 400
    assert client.post(f"/api/v1/sagas/{gid}/steps/{step_id}/execute").status_code == 400
    det = client.get(f"/api/v1/sagas/{gid}").json()
    assert det["steps"][0]["state"] == "committed"
    assert [s["saga_id"] for s in client.get(f"/api/v1/sessions/{sid}/sagas").json()] == [gid]
    assert client.get(f"/api/v1/sessions/{sid}").json()["sagas"][0]["saga_id"] == gid


def test_liability_routes(client):
    sid = _session(client)
    v = client.post(f"/api/v1/sessions/{sid}/vouch", json={"voucher_did": "did:hi", "vouchee_did": "did:lo",
                                                            "voucher_sigma": 0.9})
    assert v.status_code == 201
    assert v.json()["bonded_amount"] == pytest.approx(0.18) and v.json()["is_active"]
    bad = client.post(f"/api/v1/sessions/{sid}/vouch", json={"voucher_did": "did:x", "vouchee_did": "did:x",
                                                              "voucher_sigma": 0.9})
    assert bad.status_code == 400 and "yourself" in bad.json()["detail"]
    assert len(client.get(f"/api/v1/sessions/{sid}/vouches").json()) == 1
    lia = client.get("/api/v1/agents/did:hi/liability").json()
    assert lia["total_exposure"] == pytest.approx(0.18) and len(lia["vouches_given"]) == 1
    assert len(client.get("/api/v1/agents/did:lo/liability").json()["vouches_received"]) == 1
    assert client.get("/api/v1/stats").json()["total_vouches"] == 1


def test_events_are_recorded_and_filterable(client):
    sid = _session(client)
    client.post(f"/api/v1/sessions/{sid}/join", json={"agent_did": "did:a", "sigma_raw": 0.8})
    ev = client.get("/api/v1/events").json()
    assert ev and all(e["session_id"] == sid for e in ev)
    types = {e["event_type"] for e in ev}
    assert "session.created" in types
    only = client.get("/api/v1/events", params={"event_type": "session.created"}).json()
    assert len(only) == 1
    assert client.get("/api/v1/events", params={"event_type": "bogus"}).status_code == 400
    assert len(client.get("/api/v1/events", params={"limit": 1}).json()) == 1
    stats = client.get("/api/v1/events/stats").json()
    assert stats["total_events"] == len(ev) and stats["by_type"]["session.created"] == 1


def test_pipeline_batch_endpoint_cpu():
    """The batched pipeline endpoint writes the hypervisor's own store rows: the
    sessions are ordinary sessions, readable by id through the API and the façade."""
    from hypervisor import Hypervisor

    hv = Hypervisor(device="cpu")
    with TestClient(create_app(hv)) as client:
        r = client.post("/api/v1/engine/pipeline", json={"sessions": 256, "deltas": 3})
        assert r.status_code == 200, r.text
        body = r.json()
        assert body["completed"] == 256 and body["device"] == "cpu" and len(body["sample_merkle_root"]) == 64
        sid = body["sample_session_id"]
        d = client.get(f"/api/v1/sessions/{sid}")
        assert d.status_code == 200, d.text
        assert d.json()["state"] == "archived" and d.json()["participant_count"] == 1
        m = hv.get_session(sid)
        assert m.delta_engine.verify_chain() and m.delta_engine.compute_merkle_root() == body["sample_merkle_root"]
        assert client.get("/api/v1/stats").json()["batched_sessions"] == 256
        assert client.get("/api/v1/sessions/session:00000000-0000-4000-8000-000000000000").status_code == 404
        # later calls see the same rows: terminating an archived batch session is the reference's error
        assert client.post(f"/api/v1/sessions/{sid}/terminate").status_code == 400


def test_pipeline_batch_endpoint_on_host_engines_is_refused():
    from hypervisor import Hypervisor

    with TestClient(create_app(Hypervisor(device="host"))) as client:
        r = client.post("/api/v1/engine/pipeline", json={"sessions": 4, "deltas": 3})
        assert r.status_code == 400 and "device-backed" in r.json()["detail"]


def test_batches_stay_addressable():
    from hypervisor import Hypervisor

    hv = Hypervisor(device="cpu")
    b1 = hv.pipeline_batch(40, now_us=1767225600000000)
    b2 = hv.pipeline_batch(40, now_us=1767225601000000)  # store rows: nothing is overwritten
    for b in (b1, b2):
        for sid in (b.session_ids[0], b.session_ids[39]):
            m = hv.get_session(sid)
            assert m is not None and m.delta_engine.compute_merkle_root() == b.roots[sid]
    assert hv.get_session("not-a-session") is None


def test_dashboard_page_and_live_summary(client):
    page = client.get("/dashboard")
    assert page.status_code == 200 and "Agent Hypervisor" in page.text and "/api/v1/dashboard/summary" in page.text
    sid = _session(client)
    client.post(f"/api/v1/sessions/{sid}/join", json={"agent_did": "did:a", "sigma_raw": 0.8})
    client.post(f"/api/v1/sessions/{sid}/vouch", json={"voucher_did": "did:hi", "vouchee_did": "did:a",
                                                        "voucher_sigma": 0.9})
    client.post(f"/api/v1/sessions/{sid}/sagas")
    s = client.get("/api/v1/dashboard/summary").json()
    assert s["overview"]["sessions"] == 1 and s["overview"]["participants"] == 1
    assert s["rings"] == {"RING_2_STANDARD": 1}
    assert s["sagas"]["by_state"] == {"running": 1}
    assert s["liability"]["top_exposure"][0]["agent_did"] == "did:hi"
    assert s["events"]["recent"][0]["event_type"] in {"saga.created", "liability.vouch_created"}
    assert s["engine"] is None
    assert s["sessions"][0]["session_id"] == sid and s["agents"][0]["agent_did"] == "did:a"
    assert s["liability"]["vouches"][0]["voucher_did"] == "did:hi" and s["sagas"]["rows"][0]["state"] == "running"
    assert s["overview"]["state_authority"] in ("host", "device")
