"""Node-local RPC endpoint (agent_hypervisor_amd/parallel/rpc.py): a dropped
connection never leaves a caller waiting forever."""

from __future__ import annotations

import asyncio

import pytest

from agent_hypervisor_amd.parallel.rpc import RpcEndpoint


async def _pair():
    async def handler(name, args, kwargs):
        if name == "echo":
            return args[0]
        if name == "slow":
            await asyncio.sleep(10)
        return None

    a = RpcEndpoint(0, handler, ["echo", "slow"])
    b = RpcEndpoint(1, handler, ["echo", "slow"])
    a.peers[1] = await b.start()
    b.peers[0] = await a.start()
    return a, b


def test_call_after_the_peer_closed_the_connection_reconnects():
    async def go():
        a, b = await _pair()
        try:
            assert await a.call(1, "echo", 7) == 7
            # the server side drops every connection (a restarted or overloaded peer)
            for t in list(b._tasks):
                t.cancel()
            writer = a._conns[1][0]
            writer.transport.abort()  # the socket dies under the client
            await asyncio.sleep(0.05)
            # the next call must reconnect (or fail) — never hang on the dead writer
            got = await asyncio.wait_for(a.call(1, "echo", 8), 5)
            assert got == 8
            # send() on a peer that is not connected gives a failed future, not a pending one
            a.drop(1)
            f = a.send(1, "echo", 9)
            with pytest.raises(ConnectionError):
                await asyncio.wait_for(f, 5)
        finally:
            await a.close()
            await b.close()

    asyncio.run(go())


def test_pending_call_fails_when_its_connection_is_lost():
    async def go():
        a, b = await _pair()
        try:
            await a.connect(1)
            fut = asyncio.ensure_future(a.call(1, "slow"))
            await asyncio.sleep(0.05)
            a._conns[1][0].transport.abort()
            with pytest.raises(ConnectionError):
                await asyncio.wait_for(fut, 5)
            assert 1 not in a._conns  # the dead connection was forgotten
        finally:
            await a.close()
            await b.close()

    asyncio.run(go())


def test_create_session_on_a_dead_or_unknown_rank_is_refused_not_spun_on():
    """minting an id for a rank that is not live can never succeed (ids
    only hash to live ranks): refused at once instead of looping on the event loop."""
    from agent_hypervisor_amd.parallel.sharded import ShardedHypervisor
    from hypervisor import SessionConfig

    async def go():
        shv = await ShardedHypervisor(device="host", single=True).start()
        with pytest.raises(ValueError, match="not a live member"):
            await asyncio.wait_for(shv.create_session(SessionConfig(), "did:admin", rank=3), 5)
        sid = await shv.create_session(SessionConfig(), "did:admin", rank=0)
        assert shv.owner(sid) == 0

    asyncio.run(go())
