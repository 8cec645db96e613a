"""REST front-end of the sharded (one process per GPU) hypervisor.

Any rank may serve HTTP (typically rank 0, or one front-end per rank behind a
load balancer).  Per-session routes run on the session's owner rank — directly
when this rank owns it, otherwise forwarded point-to-point to the owner while
the other ranks keep serving (:class:`~agent_hypervisor_amd.parallel.sharded.ShardedHypervisor`);
requests are handled concurrently.  The cross-session routes combine every rank
(``/stats`` X04, ``/agents/{did}/ring`` X05, ``/agents/{did}/liability`` X01,
``/sessions``).  Ranks without a front-end run
:func:`~agent_hypervisor_amd.parallel.sharded.serve_followers`.  Error mapping
follows the single-process server (reference api/server.py): ``ValueError`` /
unknown ids → 404, other failures → 400.  The same routes, paths and request
bodies as :mod:`hypervisor.api.server` for the lifecycle, liability and saga
surfaces; the step executor of ``.../execute`` is the registered ``"noop"`` (the
reference REST executes a no-op).
"""

from __future__ import annotations

from typing import Any, Optional

from fastapi import FastAPI, HTTPException

from agent_hypervisor_amd.parallel.sharded import ShardedHypervisor
from hypervisor import __version__
from hypervisor.api.models import AddStepRequest, CreateSessionRequest, CreateVouchRequest, JoinSessionRequest
from hypervisor.models import ExecutionRing
from hypervisor.saga.state_machine import SagaStateError


def create_sharded_app(shv: ShardedHypervisor) -> FastAPI:
    from contextlib import asynccontextmanager

    @asynccontextmanager
    async def lifespan(application: FastAPI):
        if shv._stopped is None:  # the RPC endpoint lives on the serving event loop
            await shv.start()
        yield
        await shv.shutdown()
        await shv.close()

    app = FastAPI(title="Agent Hypervisor (sharded)", version=__version__, lifespan=lifespan)

    async def call(coro):
        try:
            return await coro
        except (ValueError, KeyError, SagaStateError) as e:
            raise HTTPException(status_code=404, detail=str(e)) from e
        except HTTPException:
            raise
        except Exception as e:  # noqa: BLE001
            raise HTTPException(status_code=400, detail=str(e)) from e

    @app.get("/health")
    async def health() -> dict[str, Any]:
        return {"status": "ok", "version": __version__, "world": shv.world, "rank": shv.rank}

    @app.get("/api/v1/stats")
    async def stats() -> dict[str, Any]:
        return dict(await call(shv.stats()), version=__version__, world=shv.world)

    @app.post("/api/v1/sessions", status_code=201)
    async def create_session(req: CreateSessionRequest) -> dict[str, Any]:
        sid = await call(shv.create_session(req.to_config(), req.creator_did))
        return {"session_id": sid, "rank": shv.owner(sid)}

    @app.get("/api/v1/sessions")
    async def list_sessions(state: Optional[str] = None) -> list[dict[str, Any]]:
        return await call(shv.list_sessions(state))

    @app.get("/api/v1/sessions/{session_id}")
    async def get_session(session_id: str) -> dict[str, Any]:
        return await call(shv.get_session(session_id))

    @app.post("/api/v1/sessions/{session_id}/join")
    async def join(session_id: str, req: JoinSessionRequest) -> dict[str, Any]:
        ring = await call(shv.join_session(session_id, req.agent_did, sigma_raw=req.sigma_raw,
                                           actions=req.actions or None))
        ring = ExecutionRing(ring)
        return {"agent_did": req.agent_did, "session_id": session_id, "assigned_ring": ring.value,
                "ring_name": ring.name}

    @app.post("/api/v1/sessions/{session_id}/activate")
    async def activate(session_id: str) -> dict[str, Any]:
        await call(shv.activate_session(session_id))
        return {"session_id": session_id, "state": "active"}

    @app.post("/api/v1/sessions/{session_id}/terminate")
    async def terminate(session_id: str) -> dict[str, Any]:
        root = await call(shv.terminate_session(session_id))
        return {"session_id": session_id, "state": "archived", "merkle_root": root}

    @app.get("/api/v1/agents/{agent_did}/ring")
    async def agent_ring(agent_did: str) -> dict[str, Any]:
        r = await call(shv.agent_ring(agent_did))
        if r is None:
            raise HTTPException(status_code=404, detail=f"Agent {agent_did} not found in any session")
        return dict(r, ring_name=ExecutionRing(r["ring"]).name)

    @app.post("/api/v1/sessions/{session_id}/vouch", status_code=201)
    async def vouch(session_id: str, req: CreateVouchRequest) -> dict[str, Any]:
        from datetime import datetime

        expiry = datetime.fromisoformat(req.expiry) if req.expiry else None
        return await call(shv.vouch(req.voucher_did, req.vouchee_did, session_id, req.voucher_sigma, req.bond_pct,
                                    expiry))

    @app.get("/api/v1/agents/{agent_did}/liability")
    async def liability(agent_did: str) -> dict[str, Any]:
        return await call(shv.agent_liability(agent_did))

    @app.post("/api/v1/sessions/{session_id}/sagas", status_code=201)
    async def create_saga(session_id: str) -> dict[str, Any]:
        return {"saga_id": await call(shv.create_saga(session_id)), "session_id": session_id}

    @app.get("/api/v1/sagas/{saga_id}")
    async def get_saga(saga_id: str) -> dict[str, Any]:
        return await call(shv.get_saga(saga_id))

    @app.post("/api/v1/sagas/{saga_id}/steps", status_code=201)
    async def add_step(saga_id: str, req: AddStepRequest) -> dict[str, Any]:
        sid = await call(shv.add_step(saga_id, req.action_id, req.agent_did, req.execute_api, req.undo_api,
                                      req.timeout_seconds, req.max_retries))
        return {"step_id": sid, "saga_id": saga_id}

    @app.post("/api/v1/sagas/{saga_id}/steps/{step_id}/execute")
    async def execute(saga_id: str, step_id: str) -> dict[str, Any]:
        await call(shv.execute_step(saga_id, step_id, "noop"))
        return {"saga_id": saga_id, "step_id": step_id, "state": "committed"}

    return app
