"""hipGraph capture/replay of steady-state pipeline batches (N07) and the
device time base (N09).

A steady-state governance step is a fixed launch sequence:

    clock kernel   — stamp ``cursor.now_us`` from the device wall clock
    [agent refresh] — optional caller-supplied capturable op (e.g. randint)
    pipeline kernel — full governance pipeline for ``n`` sessions, reading its
                      slot/id/time bases from ``cursor``
    advance kernel — move ``cursor`` slot/id bases past this batch
    [collective]   — optional capturable reduction of the batch counters

Captured once into a hipGraph, a step costs one ``hipGraphLaunch`` — the host
never has to compute bases or timestamps, and nothing in the loop needs a
ProcessGroup (RCCL through :class:`agent_hypervisor_amd.parallel.rccl.Communicator`
is capturable).  On CPU engines the same sequence runs eagerly through the
host twins, which keeps the semantics testable without a GPU.

Reference: the saga step loop and benchmark loop this replaces are
orchestrator.py:104-143 and bench_hypervisor.py:217-239.
"""

from __future__ import annotations

from dataclasses import dataclass
from typing import Callable, Optional

import torch

from agent_hypervisor_amd._native import C
from hypervisor import _clock


@dataclass
class DeviceClock:
    """Pairs one device wall-clock sample with host UTC microseconds."""

    base_us: int
    base_clk: int
    rate_khz: int

    @classmethod
    def calibrate(cls, device: torch.device) -> "DeviceClock":
        if device.type != "cuda":
            return cls(_clock.now_us(), 0, 1000)
        idx = device.index if device.index is not None else torch.cuda.current_device()
        torch.cuda.synchronize(device)
        rate = int(C.device_wall_clock_rate_khz(idx))
        clk = int(C.device_wall_clock(idx))
        return cls(_clock.now_us(), clk, rate)

    def stamp(self, cursor: torch.Tensor) -> None:
        """Write "now" into ``cursor[2]`` on the current stream (host twin on CPU)."""
        if cursor.device.type == "cuda":
            C.pipeline_clock(cursor.data_ptr(), self.base_us, self.base_clk, self.rate_khz,
                             torch.cuda.current_stream(cursor.device).cuda_stream)
        else:
            cursor[2] = _clock.now_us()


def advance(cursor: torch.Tensor, n: int, capacity: int) -> None:
    if cursor.device.type == "cuda":
        C.pipeline_advance(cursor.data_ptr(), n, capacity, torch.cuda.current_stream(cursor.device).cuda_stream)
    else:
        cursor[0] = (cursor[0] + n) % capacity
        cursor[1] += 3 * n


class PipelineGraph:
    """A captured governance-pipeline step for a fixed batch size.

    ``agents`` is the (device) int32 buffer of joining agent ids read by every
    replay; ``refresh_agents`` (optional, capturable) rewrites it each step.
    ``stats`` (int64[6]) receives each step's batch counters; ``reduce`` is an
    optional capturable collective applied to it (e.g. ``comm.all_reduce``);
    ``tail`` an optional capturable op run after the batch (e.g. config2's σ_eff
    and ring re-gate), so the whole step is one graph launch.

    On the GPU the step is two nodes besides the hooks: the pipeline kernel and one
    epilogue kernel that folds the counters, advances the cursor and stamps the
    next step's time base (``fused=False``: the separate zero / clock / fold /
    advance nodes).
    """

    def __init__(
        self,
        engine,
        n: int,
        agents: torch.Tensor,
        deltas: int = 3,
        stats: Optional[torch.Tensor] = None,
        refresh_agents: Optional[Callable[[], None]] = None,
        reduce: Optional[Callable[[torch.Tensor], object]] = None,
        use_graph: Optional[bool] = None,
        tail: Optional[Callable[[], None]] = None,
        fused: bool = True,
    ) -> None:
        if n > engine.sessions.capacity:
            raise ValueError(f"batch of {n} exceeds session capacity {engine.sessions.capacity}")
        if agents.numel() != n or agents.dtype != torch.int32 or agents.device != engine.device:
            raise ValueError("agents must be an int32 tensor of n ids on the engine device")
        self.engine, self.n, self.deltas = engine, n, deltas
        self.agents, self.stats = agents, stats
        self._refresh, self._reduce, self._tail = refresh_agents, reduce, tail
        dev = engine.device
        self._fused = fused and dev.type == "cuda"
        self.clock = DeviceClock.calibrate(dev)
        now = _clock.now_us()
        # [slot_base, id_base, now_us] (+ [3]: the last batch's now_us, fused epilogue)
        self.cursor = torch.tensor([engine._next_slot, engine._id_counter, now] + ([now] if self._fused else []),
                                   dtype=torch.int64, device=dev)
        self.steps = 0
        self.use_graph = (dev.type == "cuda") if use_graph is None else use_graph
        self.graph = None
        if self.use_graph:
            self._capture()

    # -- the captured body ----------------------------------------------------------
    def _body(self) -> None:
        if self._fused:
            # the cursor's time base was stamped by the previous step's epilogue
            # (or at construction): pipeline kernel + one epilogue node
            if self._refresh is not None:
                self._refresh()
            eng = self.engine
            eng.run_pipeline(self.n, agents=self.agents, deltas=self.deltas, stats=self.stats, cursor=self.cursor,
                             fold=False)
            c = self.clock
            spread = eng._spread.buf if self.stats is not None else None
            C.pipeline_epilogue(spread.data_ptr() if spread is not None else 0,
                                self.stats.data_ptr() if spread is not None else 0,
                                self.stats.numel() if spread is not None else 0, self.cursor.data_ptr(), self.n,
                                eng.sessions.capacity, c.base_us, c.base_clk, c.rate_khz,
                                torch.cuda.current_stream(self.cursor.device).cuda_stream)
        else:
            if self.stats is not None:
                self.stats.zero_()
            self.clock.stamp(self.cursor)
            if self._refresh is not None:
                self._refresh()
            self.engine.run_pipeline(self.n, agents=self.agents, deltas=self.deltas, stats=self.stats,
                                     cursor=self.cursor)
            advance(self.cursor, self.n, self.engine.sessions.capacity)
        if self._tail is not None:
            self._tail()
        if self._reduce is not None and self.stats is not None:
            self._reduce(self.stats)

    def _capture(self) -> None:
        dev = self.engine.device
        # warm up on a side stream (allocator / lazy-init work must not be captured),
        # then restore the cursor and host counters so the warm-up batch is rewritten
        saved = self.cursor.clone()
        side = torch.cuda.Stream(dev)
        side.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(side):
            self._body()
        torch.cuda.current_stream(dev).wait_stream(side)
        torch.cuda.synchronize(dev)
        self.cursor.copy_(saved)
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph):
            self._body()
        torch.cuda.synchronize(dev)

    # -- replay ---------------------------------------------------------------------
    def step(self) -> None:
        """Run one batch (graph replay on GPU, eager host twins on CPU)."""
        if self.graph is not None:
            self.graph.replay()
        else:
            self._body()
        self.steps += 1
        eng = self.engine
        # mirror the device cursor on the host so eager run_pipeline calls stay consistent
        eng._next_slot = (eng._next_slot + self.n) % eng.sessions.capacity
        eng._id_counter += 3 * self.n

    def last_batch(self):
        """Handle on the rows of the most recent step (synchronises)."""
        from agent_hypervisor_amd.models.engine import PipelineBatch

        if self.steps == 0:
            raise RuntimeError("no step has run yet")
        self.engine.synchronize()
        cur = [int(x) for x in self.cursor.cpu().tolist()]
        slot, idb = cur[0], cur[1]
        now = cur[3] if self._fused else cur[2]  # the epilogue already stamped the next step's time base
        cap = self.engine.sessions.capacity
        return PipelineBatch(self.engine, (slot - self.n) % cap, self.n, idb - 3 * self.n, now, self.deltas,
                             list(self.engine._last_specs or []), self.agents)
