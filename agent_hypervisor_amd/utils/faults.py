"""Fault injection for the kernel dispatcher.

Tests wrap a region in :class:`inject` to make named kernel launches
misbehave and check that the governance layer notices:

* ``drop``    — the launch is skipped (outputs keep stale contents);
* ``delay``   — sleep ``seconds`` before launching (slow device / straggler);
* ``corrupt`` — after the launch, flip one bit of output tensor ``target``
  (silent data corruption that the audit layer must catch).

Every launch through :func:`agent_hypervisor_amd.ops._launch.launch` consults
the active injectors; with none active the cost is one list check.
"""

from __future__ import annotations

import time
from dataclasses import dataclass, field
from typing import Optional

import torch

_ACTIVE: list["inject"] = []


@dataclass
class inject:  # noqa: N801 - used as a context manager: `with inject("hash_many", "drop"):`
    kernel: str
    mode: str
    target: Optional[str] = None
    seconds: float = 0.0
    index: int = 0
    times: Optional[int] = None
    hits: int = field(default=0, init=False)

    def __post_init__(self) -> None:
        if self.mode not in ("drop", "delay", "corrupt"):
            raise ValueError(f"unknown fault mode {self.mode!r}")
        if self.mode == "corrupt" and not self.target:
            raise ValueError("corrupt needs the name of an output tensor")

    def __enter__(self) -> "inject":
        _ACTIVE.append(self)
        return self

    def __exit__(self, *exc) -> None:
        _ACTIVE.remove(self)

    def _applies(self, name: str) -> bool:
        return name == self.kernel and (self.times is None or self.hits < self.times)


def before_launch(name: str) -> bool:
    """Return False when the launch must be dropped."""
    run = True
    for f in list(_ACTIVE):
        if not f._applies(name):
            continue
        if f.mode == "drop":
            f.hits += 1
            run = False
        elif f.mode == "delay":
            f.hits += 1
            time.sleep(f.seconds)
    return run


def after_launch(name: str, tensors: dict) -> None:
    for f in list(_ACTIVE):
        if f.mode != "corrupt" or not f._applies(name):
            continue
        t = tensors.get(f.target)
        if t is None:
            continue
        f.hits += 1
        flat = t.view(-1).view(torch.uint8) if t.dtype != torch.uint8 else t.view(-1)
        i = f.index % flat.numel()
        flat[i] ^= 1


def active() -> bool:
    return bool(_ACTIVE)
