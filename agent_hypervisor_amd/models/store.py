"""GovernanceStore: the device-authoritative state behind ``Hypervisor(device=...)``.

Every row of governance state the public API owns — sessions and their
participants, the audit chain (digests + canonical-JSON records), vouch bonds,
sagas and steps — lives in SoA PyTorch tensors on the HIP device (SURVEY N04;
column list: ``STORE_COLUMNS`` of ``csrc/include/ahv/store.h``).  API calls are
commands executed by a resident gfx950 worker wave (``csrc/hip/store_worker.hip``)
over a PCIe doorbell ring; the host keeps only what is not state: string
interning (DIDs / liability-session keys → dense ids), row allocators, and
Python objects the user handed in (executors, results, VFS file contents).

``device="cpu"`` runs the identical command processor (``store_exec``) inline on
CPU tensors — the host twin the CPU suite and the reference oracle run against.

One store per (process, device) is shared by every ``Hypervisor`` on it
(:func:`shared_store`): the reference benchmark builds a fresh ``Hypervisor()``
per pipeline, which must not allocate tables each time.  Rows are recycled ring
style when a table wraps; the default capacities (``AHV_STORE_*``) size one GPU
for ~65 k live sessions — raise them for resident populations (a session row is
≈1.1 KB with 32 participant rows; 288 GB holds >10⁸).
"""

from __future__ import annotations

import atexit
import os
import struct
import threading
from typing import Optional

import torch

from agent_hypervisor_amd._native import C
from agent_hypervisor_amd.utils.interner import Interner

OPS = dict(C.STORE_OPS)
globals().update(OPS)  # OP_* constants

_DTYPES = {
    "uint8_t": torch.uint8,
    "int32_t": torch.int32,
    "uint32_t": torch.int32,  # bit patterns (digest / uuid words)
    "int64_t": torch.int64,
    "double": torch.float64,
}

ST_OK, ST_BAD_STATE, ST_NOT_FOUND, ST_BAD_ARG, ST_SCRATCH = 0, 1, 2, 90, 91

_u64 = struct.Struct("<Q")
_d = struct.Struct("<d")


def dbits(x: float) -> int:
    """fp64 bit pattern as a signed int64 (store argument encoding)."""
    v = _u64.unpack(_d.pack(float(x)))[0]
    return v - (1 << 64) if v >= 1 << 63 else v


def bitsd(v: int) -> float:
    return _d.unpack(_u64.pack(v & 0xFFFFFFFFFFFFFFFF))[0]


def _env_int(name: str, default: int) -> int:
    v = os.environ.get(name)
    return int(v) if v else default


def default_caps() -> dict:
    return {
        "S": _env_int("AHV_STORE_SESSIONS", 1 << 16),
        "P": _env_int("AHV_STORE_PARTICIPANTS", 32),
        "D": _env_int("AHV_STORE_DELTAS", 1 << 18),
        "E": _env_int("AHV_STORE_VOUCHES", 1 << 18),
        "V": _env_int("AHV_STORE_LIABILITY_SESSIONS", 1 << 16),
        "G": _env_int("AHV_STORE_SAGAS", 1 << 16),
        "T": _env_int("AHV_STORE_STEPS", 1 << 17),
        "X": _env_int("AHV_STORE_SCRATCH", 1 << 22),
        "B": _env_int("AHV_STORE_PAYLOAD", 1 << 26),
    }


class StoreError(RuntimeError):
    """A store command failed for a reason the API layer does not map to a user error."""


class GovernanceStore:
    """Device tables + command transport + host-side allocators/interners."""

    def __init__(self, device: str = "cuda", caps: Optional[dict] = None, idle_us: Optional[int] = None) -> None:
        dev = torch.device(device)
        if dev.type == "cuda":
            if not torch.cuda.is_available():
                raise RuntimeError("GovernanceStore(device='cuda') needs a HIP device")
            if dev.index is None:
                dev = torch.device("cuda", torch.cuda.current_device())
        elif dev.type != "cpu":
            raise ValueError(f"unsupported store device {dev}")
        self.device = dev
        self.caps = dict(default_caps(), **(caps or {}))
        c = self.caps
        ext = {
            "S": c["S"], "S4": c["S"] * 4, "S8": c["S"] * 8, "SP": c["S"] * c["P"],
            "D": c["D"], "D8": c["D"] * 8, "E": c["E"], "V": c["V"], "G": c["G"], "T": c["T"], "SCR": c["X"],
        }
        self.tables: dict[str, torch.Tensor] = {}
        for name, ctype, kind in C.STORE_COLUMNS:
            fill = -1 if name in ("v_head", "v_tail", "s_dlast", "d_prev", "e_next") else 0
            self.tables[name] = torch.full((ext[kind],), fill, dtype=_DTYPES[ctype], device=dev)
        self.tables["s_state"].fill_(255)
        if dev.type == "cuda":
            torch.cuda.synchronize(dev)
        ptrs = {k: v.data_ptr() for k, v in self.tables.items()}
        self._c = C.Store(
            dev.index if dev.type == "cuda" else -1, ptrs, dict(c),
            idle_us=idle_us if idle_us is not None else _env_int("AHV_STORE_IDLE_US", 500),
        )
        self._lock = threading.RLock()
        self.agents = Interner()  # DID → dense agent id
        self.keys = Interner()  # (tenant, session id) liability keys → dense liability-session id
        self._next = {"S": 0, "E": 0, "G": 0, "T": 0}
        self._tenants = 0
        self.seed = int.from_bytes(os.urandom(8), "little") >> 1

    # -- allocation ----------------------------------------------------------
    def alloc(self, kind: str) -> int:
        """Next row of table ``kind`` (S sessions, E vouch edges, G sagas, T steps)."""
        i = self._next[kind]
        cap = self.caps[kind]
        if kind == "E" and i >= cap:
            raise StoreError(f"vouch table full ({cap} edges); raise AHV_STORE_VOUCHES")
        self._next[kind] = i + 1
        return i % cap

    def new_tenant(self) -> int:
        self._tenants += 1
        return self._tenants

    def agent_id(self, did: str) -> int:
        return self.agents.intern(did)

    def did(self, agent_id: int) -> str:
        return self.agents.str(agent_id)

    def liability_id(self, tenant: int, session_id: str) -> int:
        v = self.keys.intern(f"{tenant}\x00{session_id}")
        if v >= self.caps["V"]:
            raise StoreError(f"liability-session table full ({self.caps['V']}); raise AHV_STORE_LIABILITY_SESSIONS")
        return v

    def liability_lookup(self, tenant: int, session_id: str) -> int:
        return self.keys.lookup(f"{tenant}\x00{session_id}")

    # -- transport -----------------------------------------------------------
    def post(self, op: int, args: list, inline: Optional[bytes] = None) -> int:
        return self._c.post(op, args, inline)

    def call(self, op: int, args: list, nres: int = 4, inline: Optional[bytes] = None) -> tuple:
        return self._c.call(op, args, nres, inline)

    def result(self, seq: int, nres: int = 4) -> tuple:
        return self._c.result(seq, nres)

    def stage(self, data: bytes) -> int:
        return self._c.stage(data)

    def bulk(self, off: int, n: int) -> bytes:
        return self._c.bulk(off, n)

    def payload(self, off: int, n: int) -> bytes:
        return self._c.payload(off, n)

    def capture(self, slot: int, turn: int, ts_us: int, delta) -> tuple:
        return self._c.capture(slot, turn, ts_us, delta)

    def drain(self) -> None:
        self._c.drain()

    def flush(self) -> None:
        """Make every table write visible to other kernels / torch reads (release)."""
        self.call(OP_FLUSH, [], 1)

    def acquire(self) -> None:
        """Make rows written by other kernels (batched pipeline) visible to the worker."""
        self.call(OP_ACQUIRE, [], 1)

    def close(self) -> None:
        self._c.close()

    @property
    def is_gpu(self) -> bool:
        return self._c.gpu

    def info(self) -> dict:
        return dict(self._c.info())

    def write_rows(self, rows: dict) -> None:
        """Scatter host values into table rows: ``{column: (indices, values)}``.

        Used by checkpoint restore and by host-side bulk loads.  The worker's
        dirty lines are written back first (release) and it re-reads the rows
        afterwards (acquire), so the tensor writes and the command stream agree.
        """
        self.drain()
        cuda = self.device.type == "cuda"
        if cuda:
            self.flush()
        for col, (idx, vals) in rows.items():
            if not len(idx):
                continue
            last = dict(zip(idx, vals))  # a later write to the same row wins (deterministically)
            idx, vals = list(last.keys()), list(last.values())
            t = self.tables[col]
            if t.dtype == torch.int32:
                vals = [v - (1 << 32) if v >= 1 << 31 else v for v in vals]
            t[torch.tensor(idx, dtype=torch.int64, device=self.device)] = torch.tensor(vals, dtype=t.dtype).to(
                self.device)
        if cuda:
            torch.cuda.synchronize(self.device)
            self.acquire()

    def payload_append(self, data: bytes) -> int:
        return self._c.payload_append(data)

    def alloc_delta(self) -> int:
        return self._c.alloc_delta()

    def column(self, name: str) -> torch.Tensor:
        """A table column (flushes pending device writes first)."""
        self.drain()
        if self.device.type == "cuda":
            self.flush()
        return self.tables[name]

    # -- index lists -----------------------------------------------------------
    def index_args(self, idx: list) -> tuple:
        """(count, staging offset, inline bytes) for an int32 index list argument."""
        n = len(idx)
        raw = struct.pack(f"<{n}i", *idx)
        if n <= 96:
            return n, 0, raw
        return n, self.stage(raw), None


_STORES: dict = {}
_STORES_LOCK = threading.Lock()


def shared_store(device: str) -> GovernanceStore:
    """The process-wide store of ``device`` (created on first use)."""
    key = str(torch.device(device))
    st = _STORES.get(key)
    if st is None:
        with _STORES_LOCK:
            st = _STORES.get(key)
            if st is None:
                st = GovernanceStore(device)
                _STORES[key] = st
    return st


@atexit.register
def _close_all() -> None:
    for st in list(_STORES.values()):
        try:
            st.close()
        except Exception:
            pass
