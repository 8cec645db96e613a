"""Loader for the native core ``agent_hypervisor_amd._C``.

The extension is required: there is no pure-Python fallback for the audit hash
path or for the gfx950 kernels.  If the shared object is missing or stale it is
(re)built in-tree with hipcc on first import (a few seconds per translation unit),
and any failure is raised loudly.
"""

from __future__ import annotations

import importlib
import os
import threading

_lock = threading.Lock()
_C = None


def load():
    """Return the ``_C`` extension module, building it if needed."""
    global _C
    if _C is not None:
        return _C
    with _lock:
        if _C is not None:
            return _C
        from agent_hypervisor_amd.utils import build as _build

        if os.environ.get("AHV_SKIP_AUTOBUILD") != "1" and _build.needs_build():
            _build.build()
        # torch-ROCm ships its own libamdhip64 / libhsa-runtime64 / librccl.  Load
        # them first so the extension's NEEDED sonames bind to the *same* runtime
        # objects torch uses; importing _C first would pull a second HIP runtime
        # from /opt/rocm (and a second RCCL that sees no devices).
        import torch  # noqa: F401

        _C = importlib.import_module("agent_hypervisor_amd._C")
        return _C


C = load()
