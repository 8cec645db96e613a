"""``Engine(device=...)`` → the engine's device-resident variant.

The stand-alone governance engines take an optional ``device``: without it they
are the plain host engines of the reference; with it, construction returns the
subclass in :mod:`hypervisor._device_engines` that keeps the engine's state in
device columns and runs its batched kernel.
"""

from __future__ import annotations


def device_variant(cls, host_cls, name: str, device):
    if device is not None and cls is host_cls:
        import hypervisor._device_engines as _de

        cls = getattr(_de, name)
    return object.__new__(cls)
