"""Launcher for the batched governance pipeline kernel (``csrc/hip/pipeline.hip``).

``run(args)`` validates that every tensor argument lives on one device and then
launches the gfx950 kernel on the current HIP stream — or, for CPU tensors, runs
the host twin (the same ``pipeline_session`` body instantiated for the CPU; used
by the CPU test-suite and as the reference in GPU equivalence tests).  There is
no silent fallback: a CUDA tensor always takes the kernel path.
"""

from __future__ import annotations

import torch

from agent_hypervisor_amd._native import C
from agent_hypervisor_amd.utils import faults as _faults


def run(scalars: dict, tensors: dict[str, torch.Tensor | None]) -> None:
    devs = {t.device for t in tensors.values() if t is not None}
    if len(devs) != 1:
        raise ValueError(f"pipeline tensors span devices {devs}")
    (dev,) = devs
    args = dict(scalars)
    for k, t in tensors.items():
        if t is None:
            args[k] = None
            continue
        if not t.is_contiguous():
            raise ValueError(f"pipeline argument {k} must be contiguous")
        args[k] = t.data_ptr()
    if _faults.active() and not _faults.before_launch("pipeline"):
        return  # injected fault: launch dropped
    if dev.type == "cuda":
        C.pipeline(args, torch.cuda.current_stream(dev).cuda_stream)
    elif dev.type == "cpu":
        C.pipeline_host(args)
    else:
        raise ValueError(f"unsupported device {dev}")
    if _faults.active():
        _faults.after_launch("pipeline", tensors)
