"""Common launcher for the batched kernels of ``agent_hypervisor_amd._C``.

Every kernel ``k`` is exported twice by the extension: ``k(args, stream)``
launches the gfx950 kernel on a HIP stream and ``k_host(args)`` runs the same
element body on the CPU.  :func:`launch` picks by the device of the tensor
arguments — all of which must live on one device — so CUDA tensors always take
the kernel path (no silent fallback) and CPU tensors the host twin (tests,
reference results).  Tensors must be contiguous and of the declared dtype.
"""

from __future__ import annotations

from typing import Optional

import torch

from agent_hypervisor_amd._native import C
from agent_hypervisor_amd.utils import faults as _faults


def _check(name: str, key: str, t: torch.Tensor, dtype: Optional[torch.dtype]) -> None:
    if dtype is not None and t.dtype != dtype:
        raise TypeError(f"{name}: argument {key} must be {dtype}, got {t.dtype}")
    if not t.is_contiguous():
        raise ValueError(f"{name}: argument {key} must be contiguous")


def launch(name: str, scalars: dict, tensors: dict, dtypes: Optional[dict] = None) -> torch.device:
    dtypes = dtypes or {}
    devs = {t.device for t in tensors.values() if t is not None}
    if len(devs) > 1:
        raise ValueError(f"{name}: tensors span devices {devs}")
    dev = next(iter(devs)) if devs else torch.device("cpu")
    args = dict(scalars)
    for k, t in tensors.items():
        if t is None:
            args[k] = None
            continue
        _check(name, k, t, dtypes.get(k))
        args[k] = t.data_ptr()
    if _faults.active() and not _faults.before_launch(name):
        return dev  # injected fault: launch dropped
    if dev.type == "cuda":
        getattr(C, name)(args, torch.cuda.current_stream(dev).cuda_stream)
    elif dev.type == "cpu":
        getattr(C, name + "_host")(args)
    else:
        raise ValueError(f"{name}: unsupported device {dev}")
    if _faults.active():
        _faults.after_launch(name, tensors)
    return dev


def empty_like_dev(ref: torch.Tensor, shape, dtype) -> torch.Tensor:
    return torch.empty(shape, dtype=dtype, device=ref.device)


def zeros_like_dev(ref: torch.Tensor, shape, dtype) -> torch.Tensor:
    return torch.zeros(shape, dtype=dtype, device=ref.device)
