"""Control-plane RPC between the ranks of one node, for rank-local serving.

Session-sharded serving needs *no* communication on the
per-session path when a request arrives at the session's owner rank; a request
that arrives at another rank is forwarded point-to-point to the owner, which
answers while every other rank keeps serving its own traffic.  Collectives (RCCL
over xGMI on MI355X, gloo on CPU) stay on the data plane for the agent-global
views.

Transport and safety:

* Each rank listens on a **Unix domain socket** inside a private directory
  (mode 0700, created by the rank) whose path it publishes in the process
  group's key-value store; only processes of the same user on the same node can
  connect.  The 8 GPUs of one MI355X node are one node.
* Messages are **JSON** — data only: method name, positional/keyword arguments
  made of JSON values, a result, or an error (exception class *name* + message).
  Nothing received is ever unpickled or executed.
* Only the method names in the endpoint's ``allowed`` set are dispatched; an
  error is re-raised on the caller only as one of a fixed set of exception
  classes (:data:`ERRORS`), anything else becomes :class:`RemoteError`.
"""

from __future__ import annotations

import asyncio
import itertools
import json
import os
import struct
import tempfile
from typing import Any, Awaitable, Callable, Iterable, Optional

_LEN = struct.Struct("<I")
MAX_FRAME = 64 << 20


class RemoteError(RuntimeError):
    """A remote call failed with an error that is not in :data:`ERRORS`."""


def _error_classes() -> dict:
    from hypervisor.liability.vouching import VouchingError
    from hypervisor.saga.orchestrator import SagaTimeoutError
    from hypervisor.saga.state_machine import SagaStateError
    from hypervisor.session import SessionLifecycleError, SessionParticipantError
    from hypervisor.session.sso import VFSPermissionError

    return {c.__name__: c for c in (
        ValueError, KeyError, TypeError, LookupError, RuntimeError, TimeoutError, PermissionError,
        FileNotFoundError, VouchingError, SagaStateError, SagaTimeoutError, SessionLifecycleError,
        SessionParticipantError, VFSPermissionError,
    )}


ERRORS: dict = {}


def _raise_remote(name: str, msg: str) -> None:
    if not ERRORS:
        ERRORS.update(_error_classes())
    cls = ERRORS.get(name)
    if cls is KeyError:
        raise KeyError(msg)
    raise (cls(msg) if cls is not None else RemoteError(f"{name}: {msg}"))


async def _read_frame(reader: asyncio.StreamReader) -> bytes:
    n = _LEN.unpack(await reader.readexactly(4))[0]
    if n > MAX_FRAME:
        raise ConnectionError(f"RPC frame of {n} bytes exceeds the limit")
    return await reader.readexactly(n)


def _frame(obj: Any) -> bytes:
    b = json.dumps(obj, separators=(",", ":")).encode()
    return _LEN.pack(len(b)) + b


class RpcEndpoint:
    """One rank's RPC server plus its client connections to the other ranks.

    ``handler(name, args, kwargs)`` executes an incoming call (a coroutine) for
    a name in ``allowed``; each request runs as its own task, so a slow call does
    not hold up the next.  ``counters`` counts calls in and out."""

    def __init__(self, rank: int, handler: Callable[[str, list, dict], Awaitable[Any]],
                 allowed: Iterable[str]) -> None:
        self.rank = rank
        self.handler = handler
        self.allowed = frozenset(allowed)
        self.server = None
        self.address: Optional[str] = None
        self._dir: Optional[str] = None
        self.peers: dict[int, str] = {}
        self._conns: dict[int, tuple] = {}  # rank → (writer, pending futures, reader task)
        self._ids = itertools.count(1)
        self._conn_lock: dict[int, asyncio.Lock] = {}
        self.counters = {"rpc_out": 0, "rpc_in": 0}
        self._tasks: set = set()

    async def start(self) -> str:
        self._dir = tempfile.mkdtemp(prefix="ahv-rpc-")  # 0700: only this user can reach the socket
        path = os.path.join(self._dir, f"rank{self.rank}.sock")
        self.server = await asyncio.start_unix_server(self._serve_conn, path=path)
        self.address = path
        return path

    async def close(self) -> None:
        for r in list(self._conns):
            self.drop(r)
        if self.server is not None:
            self.server.close()
            await self.server.wait_closed()
            self.server = None
        if self._dir is not None:
            for f in os.listdir(self._dir):
                os.unlink(os.path.join(self._dir, f))
            os.rmdir(self._dir)
            self._dir = None

    def drop(self, rank: int) -> None:
        """Forget a peer (a failed rank): its pending calls fail."""
        c = self._conns.pop(rank, None)
        self.peers.pop(rank, None)
        if c is not None:
            c[2].cancel()
            c[0].close()
            for f in c[1].values():
                if not f.done():
                    f.set_exception(ConnectionError(f"rank {rank} is gone"))

    # -- server side ------------------------------------------------------------
    async def _serve_conn(self, reader: asyncio.StreamReader, writer: asyncio.StreamWriter) -> None:
        try:
            while True:
                try:
                    raw = await _read_frame(reader)
                except (asyncio.IncompleteReadError, ConnectionError):
                    return
                t = asyncio.get_running_loop().create_task(self._one(raw, writer))
                self._tasks.add(t)
                t.add_done_callback(self._tasks.discard)
        finally:
            writer.close()

    async def _one(self, raw: bytes, writer: asyncio.StreamWriter) -> None:
        rid = None
        try:
            msg = json.loads(raw)
            rid, name, args, kwargs = msg["id"], msg["m"], msg.get("a", []), msg.get("k", {})
            if name not in self.allowed or not isinstance(args, list) or not isinstance(kwargs, dict):
                raise PermissionError(f"RPC method {name!r} is not served")
            self.counters["rpc_in"] += 1
            out = {"id": rid, "ok": await self.handler(name, args, kwargs)}
        except Exception as e:  # noqa: BLE001 - re-raised (by class name) on the caller
            out = {"id": rid, "err": type(e).__name__, "msg": str(e.args[0]) if isinstance(e, KeyError) and e.args
                   else str(e)}
        try:
            data = _frame(out)
        except (TypeError, ValueError) as e:
            data = _frame({"id": rid, "err": "TypeError", "msg": f"result is not JSON-serialisable: {e}"})
        writer.write(data)
        await writer.drain()

    # -- client side ------------------------------------------------------------
    async def _conn(self, rank: int):
        c = self._live(rank)
        if c is not None:
            return c
        lock = self._conn_lock.setdefault(rank, asyncio.Lock())
        async with lock:
            c = self._live(rank)
            if c is not None:
                return c
            path = self.peers.get(rank)
            if path is None:
                raise ConnectionError(f"no RPC address for rank {rank}")
            reader, writer = await asyncio.open_unix_connection(path)
            pend: dict[int, asyncio.Future] = {}
            task = asyncio.get_running_loop().create_task(self._reader(rank, reader, writer, pend))
            c = (writer, pend, task)
            self._conns[rank] = c
            return c

    def _live(self, rank: int):
        """The open connection to ``rank`` or None; a connection whose writer is
        closing is forgotten here (its reader fails its pending calls), so the
        next :meth:`call` reconnects instead of writing into a dead socket."""
        c = self._conns.get(rank)
        if c is not None and c[0].is_closing():
            self._forget(rank, c)
            return None
        return c

    def _forget(self, rank: int, c: tuple) -> None:
        if self._conns.get(rank) is c:
            del self._conns[rank]
        c[0].close()
        for f in c[1].values():
            if not f.done():
                f.set_exception(ConnectionError(f"rank {rank}: connection lost"))
        c[1].clear()

    async def _reader(self, rank: int, reader: asyncio.StreamReader, writer, pend: dict) -> None:
        try:
            while True:
                msg = json.loads(await _read_frame(reader))
                f = pend.pop(msg.get("id"), None)
                if f is None or f.done():
                    continue
                if "err" in msg:
                    try:
                        _raise_remote(str(msg["err"]), str(msg.get("msg", "")))
                    except Exception as e:  # noqa: BLE001
                        f.set_exception(e)
                else:
                    f.set_result(msg.get("ok"))
        except (asyncio.IncompleteReadError, ConnectionError, asyncio.CancelledError, ValueError, OSError):
            pass
        # the connection is dead: fail what waits on it and drop it (if it is still the
        # registered one), so later calls reconnect rather than reuse a closed writer
        c = self._conns.get(rank)
        if c is not None and c[0] is writer:
            self._forget(rank, c)
        else:
            writer.close()
            for f in pend.values():
                if not f.done():
                    f.set_exception(ConnectionError(f"rank {rank}: connection lost"))
            pend.clear()

    async def connect(self, rank: int) -> None:
        """Open the connection to ``rank`` now (so :meth:`send` can write at once)."""
        await self._conn(rank)

    def send(self, rank: int, name: str, *args, **kwargs) -> "asyncio.Future":
        """Write a call to an already connected peer *now* (no await before the bytes
        leave) and return the future of its result.  A peer whose connection is gone
        yields an already-failed future (never one that stays unresolved)."""
        fut = asyncio.get_running_loop().create_future()
        c = self._live(rank)
        if c is None:
            fut.set_exception(ConnectionError(f"rank {rank}: not connected"))
            return fut
        writer, pend, _ = c
        rid = next(self._ids)
        pend[rid] = fut
        writer.write(_frame({"id": rid, "m": name, "a": list(args), "k": kwargs}))
        self.counters["rpc_out"] += 1
        return fut

    async def call(self, rank: int, name: str, *args, **kwargs) -> Any:
        """Run ``name(*args, **kwargs)`` on ``rank`` (JSON arguments); its error is re-raised here."""
        writer, pend, _ = await self._conn(rank)
        rid = next(self._ids)
        fut = asyncio.get_running_loop().create_future()
        pend[rid] = fut
        writer.write(_frame({"id": rid, "m": name, "a": list(args), "k": kwargs}))
        self.counters["rpc_out"] += 1
        try:
            await writer.drain()
        except (ConnectionError, OSError) as e:
            pend.pop(rid, None)
            raise ConnectionError(f"rank {rank}: connection lost") from e
        return await fut
