"""Launcher for the batched template pipeline over a store's rows
(``csrc/hip/store_template.hip``, body ``csrc/include/ahv/store_template.h``).

``run(store, args, tensors)`` launches the gfx950 kernel on the current HIP
stream for a device store, or runs the host twin (the same ``template_session``
body instantiated for the CPU) for a CPU store — no silent fallback: a device
store always takes the kernel path.  The launch goes through the fault-injection
hooks (:mod:`agent_hypervisor_amd.utils.faults`) under the name ``"pipeline"``;
``tensors`` names the outputs an injected ``corrupt`` fault may flip.
"""

from __future__ import annotations

import torch

from agent_hypervisor_amd.utils import faults as _faults


def run(store, args: dict, tensors: dict[str, torch.Tensor] | None = None) -> None:
    if _faults.active() and not _faults.before_launch("pipeline"):
        return  # injected fault: launch dropped
    dev = store.device
    if dev.type == "cuda":
        store._c.run_template(args, torch.cuda.current_stream(dev).cuda_stream)
    else:
        store._c.run_template(args, 0)
    if _faults.active():
        _faults.after_launch("pipeline", tensors or {})
