"""Failure detection and session failover for session-sharded ranks.

The reference has no process-failure handling (it is a single process).  With
sessions sharded one-rank-per-GPU, a lost rank orphans its sessions; this
module provides the three pieces the rebuild plan calls for:

* :class:`Heartbeat` — every rank stamps ``hb/<rank>`` in the process group's
  key-value store; :meth:`Heartbeat.dead_ranks` reports ranks whose stamp is
  stale.  Works over any backend (the store is the rendezvous TCPStore).
* :func:`guarded` — run a torch.distributed collective asynchronously and wait
  with a deadline; :class:`CommWatchdog` polls a direct RCCL communicator's
  asynchronous error state and aborts it (so pending collectives are cancelled,
  not waited on forever) when a peer fails.
* :func:`failover_plan` / :func:`apply_failover` — re-home the failed rank's
  sessions on the survivors (least-loaded first) in the
  :class:`~agent_hypervisor_amd.parallel.directory.SessionDirectory`; their state
  is re-hydrated from the failed rank's last checkpoint
  (:mod:`agent_hypervisor_amd.runtime.checkpoint`), whose audit chains are
  re-verified on load, so Merkle chains continue from the persisted last hash.
"""

from __future__ import annotations

import threading
import time
from datetime import timedelta
from typing import Callable, Optional

import torch.distributed as dist

from agent_hypervisor_amd.parallel.directory import SessionDirectory


def _store():
    if not dist.is_initialized():
        raise RuntimeError("heartbeats need an initialised process group")
    return dist.distributed_c10d._get_default_store()


class Heartbeat:
    """Periodic liveness stamps in the process group's store."""

    def __init__(self, interval_s: float = 1.0, prefix: str = "ahv/hb") -> None:
        self.interval = interval_s
        self.prefix = prefix
        self.rank = dist.get_rank()
        self.world = dist.get_world_size()
        self._stop = threading.Event()
        self._thread: Optional[threading.Thread] = None

    def beat(self) -> None:
        _store().set(f"{self.prefix}/{self.rank}", repr(time.time()))

    def start(self) -> "Heartbeat":
        self.beat()

        def loop():
            while not self._stop.wait(self.interval):
                try:
                    self.beat()
                except Exception:  # noqa: BLE001 - store gone: the job is ending
                    return

        self._thread = threading.Thread(target=loop, name="ahv-heartbeat", daemon=True)
        self._thread.start()
        return self

    def stop(self) -> None:
        self._stop.set()
        if self._thread is not None:
            self._thread.join(timeout=5)

    def last_seen(self, rank: int) -> Optional[float]:
        key = f"{self.prefix}/{rank}"
        st = _store()
        if not st.check([key]):
            return None
        return float(st.get(key).decode())

    def dead_ranks(self, timeout_s: float) -> list[int]:
        """Ranks with no stamp, or a stamp older than ``timeout_s`` seconds."""
        now = time.time()
        dead = []
        for r in range(self.world):
            t = self.last_seen(r)
            if t is None or now - t > timeout_s:
                dead.append(r)
        return dead


def guarded(op: Callable[..., object], *args, timeout_s: float = 30.0, **kwargs) -> bool:
    """Run ``op(*args, async_op=True, **kwargs)`` (a torch.distributed
    collective) and wait at most ``timeout_s``; False on timeout or error."""
    try:
        work = op(*args, async_op=True, **kwargs)
        return bool(work.wait(timeout=timedelta(seconds=timeout_s)))
    except Exception:  # noqa: BLE001 - a failed peer surfaces as a backend error
        return False


class CommWatchdog:
    """Polls a :class:`~agent_hypervisor_amd.parallel.rccl.Communicator` for
    asynchronous errors; on one, aborts it and calls ``on_failure(message)``."""

    def __init__(self, comm, on_failure: Optional[Callable[[str], None]] = None, interval_s: float = 0.5) -> None:
        self.comm = comm
        self.on_failure = on_failure
        self.interval = interval_s
        self.failure: Optional[str] = None
        self._stop = threading.Event()
        self._thread: Optional[threading.Thread] = None

    def check(self) -> Optional[str]:
        err = self.comm.async_error()
        if err and self.failure is None:
            self.failure = err
            self.comm.abort()
            if self.on_failure is not None:
                self.on_failure(err)
        return self.failure

    def start(self) -> "CommWatchdog":
        def loop():
            while not self._stop.wait(self.interval):
                if self.check():
                    return

        self._thread = threading.Thread(target=loop, name="ahv-comm-watchdog", daemon=True)
        self._thread.start()
        return self

    def stop(self) -> None:
        self._stop.set()
        if self._thread is not None:
            self._thread.join(timeout=5)


def failover_plan(directory: SessionDirectory, failed: list[int]) -> list[tuple[str, int, int]]:
    """Moves (session, failed_rank, survivor) re-homing every session of the
    failed ranks on the least-loaded survivors."""
    survivors = [r for r in range(directory.world) if r not in set(failed)]
    if not survivors:
        raise RuntimeError("no surviving rank to fail over to")
    load = {r: directory.load[r] for r in survivors}
    moves = []
    for f in failed:
        for s in sorted(directory.sessions_of(f)):
            dst = min(survivors, key=lambda r: (load[r], r))
            moves.append((s, f, dst))
            load[dst] += 1
    return moves


def apply_failover(directory: SessionDirectory, moves: list[tuple[str, int, int]],
                   failed: Optional[list[int]] = None) -> None:
    """Re-home the moved sessions and mark the failed ranks dead, so placement
    and rebalancing never target them again (until :meth:`mark_alive`)."""
    dead = set(failed or []) | {src for _, src, _ in moves}
    if dead:
        directory.mark_dead(sorted(dead))
    directory.apply(moves)


def rehydrate(checkpoint_dir: str, moves: list[tuple[str, int, int]], rank: int, hv=None):
    """Load the sessions ``moves`` assigns to ``rank`` from the failed rank's
    checkpoint into ``hv`` (a Hypervisor, host or device-backed) through the
    checkpoint loader, which re-verifies their audit chains and roots."""
    from agent_hypervisor_amd.runtime.checkpoint import load_hypervisor

    mine = sorted({s for s, _, dst in moves if dst == rank})
    if hv is None:
        from hypervisor import Hypervisor

        hv = Hypervisor()
    return load_hypervisor(checkpoint_dir, hv=hv, sessions=mine)
