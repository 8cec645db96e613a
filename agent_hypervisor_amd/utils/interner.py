"""String interner with a device-resident mirror.

Wraps the native :class:`agent_hypervisor_amd._C.StringPool`: every DID, path,
content hash, id string … gets a dense ``int32`` id; its canonical-JSON escaped
body is stored contiguously so device kernels splice it into audit payloads.
``device_view(device)`` returns ``(bytes u8[N], offsets i64[M], lengths i32[M])``
tensors, re-uploaded only when new strings were interned since the last call.
"""

from __future__ import annotations

from typing import Iterable

import torch

from agent_hypervisor_amd._native import C


class Interner:
    def __init__(self) -> None:
        self._pool = C.StringPool()
        self._uploaded: dict[str, tuple[int, tuple[torch.Tensor, torch.Tensor, torch.Tensor]]] = {}

    # Python strings may hold lone surrogates (json.dumps escapes them as \udXXX);
    # they have no strict UTF-8 form, so such strings cross to the native pool in
    # surrogatepass UTF-8, which the native escaper decodes to the same code point.
    @staticmethod
    def _b(s: str) -> bytes:
        return s.encode("utf-8", "surrogatepass")

    def intern(self, s: str) -> int:
        try:
            return self._pool.intern(s)
        except TypeError:
            return self._pool.intern(self._b(s))

    def intern_many(self, items: Iterable[str]) -> list[int]:
        items = list(items)
        try:
            return self._pool.intern_many(items)
        except TypeError:
            return self._pool.intern_many([self._b(s) for s in items])

    def lookup(self, s: str) -> int:
        try:
            return self._pool.lookup(s)
        except TypeError:
            return self._pool.lookup(self._b(s))

    def str(self, i: int) -> str:
        return self._pool.str(int(i)).decode("utf-8", "surrogatepass")

    def escaped(self, i: int) -> bytes:
        return self._pool.escaped(int(i))

    def __len__(self) -> int:
        return len(self._pool)

    def device_view(self, device) -> tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
        key = str(device)
        n = len(self._pool)
        hit = self._uploaded.get(key)
        if hit is not None and hit[0] == n:
            return hit[1]
        raw = bytes(self._pool.bytes_view()) or b"\0"
        b = torch.frombuffer(bytearray(raw), dtype=torch.uint8)
        o = torch.frombuffer(bytearray(bytes(self._pool.offsets_view()) or b"\0" * 8), dtype=torch.int64)
        ln = torch.frombuffer(bytearray(bytes(self._pool.lengths_view()) or b"\0" * 4), dtype=torch.int32)
        view = (b.to(device), o.to(device), ln.to(device))
        self._uploaded[key] = (n, view)
        return view
