"""Whole-session migration between ranks.

Under session sharding every session has one owner rank.  Moving sessions —
rebalancing a skewed job, or emptying a rank before it leaves — moves *all* of a
session's state from one store to another:

* the session row and its participant rows, the delta chain (rows + digests) with
  the canonical-JSON records from the payload arena, sagas and steps — packed on
  the sender's device by :func:`agent_hypervisor_amd.runtime.store_checkpoint.collect`
  (one gather per column, one record-move kernel for the arena) into a single
  uint8 device buffer per destination;
* vouch edges of the session's liability list, commitments held on the host,
  VFS / reversibility extras, string ids (dictionary-encoded) — the host part.

Exchange (:func:`exchange`): one ``all_to_all_single`` of the per-destination
sizes and one of the host parts on the control group (gloo), and one
``all_to_all_single`` of the device buffers on the data group — RCCL over xGMI on
MI355X, so the bulk state (columns, digests, records) moves device to device and
never through host memory.  The receiver allocates rows, writes every column with
``index_copy_`` from the received device buffer (row references and agent ids
rewritten on the device), writes the records into its arena with the same kernel,
re-verifies every chain (K10) and committed root (K09) on the device, and registers
the sessions lazily (:class:`~agent_hypervisor_amd.runtime.store_checkpoint.RestoredBatch`).
The sender then drops them (:func:`evict`): rows returned to its store, views
detached, vouch records and liability rows released.

Reference: the reference has one process and one ``_sessions`` map
(``src/hypervisor/core.py:92-103``); a moved session answers every API call on
its new owner exactly as it did before the move.
"""

from __future__ import annotations

import json
import struct
import numpy as np
import torch
import torch.distributed as dist

from agent_hypervisor_amd.runtime import store_checkpoint as SC

_MAGIC = b"AHVM"


# ---------------------------------------------------------------- pack / unpack


def pack(hv, session_ids: list) -> tuple:
    """``(device buffer uint8, host bytes)`` holding the sessions ``session_ids`` of
    the device-backed ``hv`` (their vouches, commitments and extras included)."""
    from safetensors.torch import save

    cols, host, arena, meta = SC.collect(hv, only=set(session_ids), device=True)
    dev = hv._store.device
    layout, parts, off = [], [], 0
    for k in sorted(cols):
        t = cols[k].contiguous()
        b = t.view(torch.uint8).reshape(-1) if t.numel() else torch.zeros(0, dtype=torch.uint8, device=dev)
        layout.append([k, str(t.dtype).replace("torch.", ""), list(t.shape), off, int(b.numel())])
        parts.append(b)
        off += int(b.numel())
        pad = -off % 8  # every column starts 8-byte aligned (viewed back as int64 / fp64)
        if pad:
            parts.append(torch.zeros(pad, dtype=torch.uint8, device=dev))
            off += pad
    a = arena if isinstance(arena, torch.Tensor) else torch.zeros(0, dtype=torch.uint8, device=dev)
    layout.append(["__arena__", "uint8", [int(a.numel())], off, int(a.numel())])
    parts.append(a.to(dev))
    buf = torch.cat(parts) if parts else torch.zeros(0, dtype=torch.uint8, device=dev)
    head = json.dumps({"meta": meta, "layout": layout}).encode()
    host_bytes = _MAGIC + struct.pack("<Q", len(head)) + head + save(dict(host))
    return buf, host_bytes


_DT = {"uint8": torch.uint8, "int32": torch.int32, "int64": torch.int64, "float64": torch.float64}


def unpack(hv, buf: torch.Tensor, host_bytes: bytes, verify: str = "device"):
    """Register the sessions of one :func:`pack` (received ``buf`` on this rank's
    store device) with ``hv``; returns the restored batch."""
    from safetensors.torch import load

    if host_bytes[:4] != _MAGIC:
        raise ValueError("not a session-migration image")
    (hl,) = struct.unpack_from("<Q", host_bytes, 4)
    head = json.loads(host_bytes[12:12 + hl].decode())
    host = load(host_bytes[12 + hl:])
    dev = hv._store.device
    buf = buf.to(dev)
    cols, arena = {}, None
    for name, dt, shape, off, nb in head["layout"]:
        piece = buf[off:off + nb]
        if name == "__arena__":
            arena = piece.contiguous()
            continue
        t = piece.view(_DT[dt]) if nb else torch.zeros(0, dtype=_DT[dt], device=dev)
        cols[name] = t.reshape(shape)
    SC.restore(hv, cols, host, arena, head["meta"], verify=verify)
    return hv._sessions.batch_of(SC._Col(host, "session_id").all()[0]) if head["meta"]["sessions"] else None


# ---------------------------------------------------------------- sender side


def evict(hv, session_ids: list) -> int:
    """Drop sessions that now live on another rank: their rows return to this
    store, their views are detached, their vouch records and liability rows go.
    Returns the number of sessions dropped."""
    from hypervisor import _device

    st = hv._store
    ids = set(session_ids)
    n = 0
    saga_rows = []
    for sid in ids:
        batch = hv._sessions.batch_of(sid)
        m = hv._sessions.pop(sid)  # own: its views; batch: the built view, or None (unbuilt: dropped)
        if m is None and batch is None:
            continue
        n += 1
        if m is not None:
            if isinstance(m.saga, _device.DeviceSagaOrchestrator):
                saga_rows.extend(g.slot for g in m.saga._sagas.values())
            if isinstance(m.sso, _device.DeviceSession):
                _device._close_views(st, m)
        ce = hv.commitment
        getattr(ce, "_device", {}).pop(sid, None)
        getattr(ce, "_commitments", {}).pop(sid, None)
    # unbuilt batch sessions dropped above: released now — every batch, including one
    # this eviction emptied (segments() no longer lists it, its dead rows still wait)
    for seg in hv._sessions.batches():
        if seg.dead:
            seg.release(np.asarray(seg.dead, dtype=np.int64))
            seg.dead = []
    hv._sessions.prune_batches()
    hv._sessions.forget_sagas(saga_rows)
    _evict_vouches(hv, ids)
    return n


def _evict_vouches(hv, ids: set) -> None:
    from hypervisor import _device

    ve = hv.vouching
    if not isinstance(ve, _device.DeviceVouchingEngine):
        return
    st = hv._store
    gone = [r for r in ve._order if r.session_id in ids]
    if not gone:
        return
    edges = []
    for r in gone:
        ve._by_id.pop(r.vouch_id, None)
        e = getattr(r, "edge", -1)
        if e >= 0 and ve._by_edge.pop(e, None) is not None:
            edges.append(e)
            r.__dict__["_store"] = _device.CLOSED
    ve._order = [r for r in ve._order if r.session_id not in ids]
    if edges:
        st.release_many("E", edges)
    tv = st._tenant_v.get(ve._tenant, {})
    vrows = [tv.pop(s) for s in list(ids) if s in tv]
    if vrows:
        st.release_many("V", vrows)


# ---------------------------------------------------------------- exchange


def exchange(hv, plan: dict, rank: int, members: list, ctrl_group=None, data_group=None,
             verify: str = "device") -> list:
    """Collective over ``members`` (sorted global ranks; the groups' rank order):
    send ``plan[dst]`` (session ids this rank owns) to each ``dst`` and register
    what the others send here.  Returns the session ids received.  Bulk state moves
    in one ``all_to_all_single`` on ``data_group`` (device buffers); sizes and
    host parts on ``ctrl_group``."""
    st = hv._store
    dev = st.device
    nccl = dist.get_backend(data_group) == "nccl" if data_group is not None else dist.get_backend() == "nccl"
    data_dev = dev if nccl else torch.device("cpu")
    k = len(members)
    bufs: list = [None] * k
    hosts: list = [b""] * k
    for j, dst in enumerate(members):
        sids = plan.get(dst)
        if dst != rank and sids:
            bufs[j], hosts[j] = pack(hv, list(sids))
    sizes = torch.tensor([[len(hosts[j]), int(bufs[j].numel()) if bufs[j] is not None else 0] for j in range(k)],
                         dtype=torch.int64).reshape(-1)
    rsizes = torch.empty(2 * k, dtype=torch.int64)
    dist.all_to_all_single(rsizes, sizes, group=ctrl_group)
    s_out, r_in = sizes.view(k, 2), rsizes.view(k, 2)
    # host parts (gloo, CPU)
    hsend = torch.frombuffer(bytearray(b"".join(hosts)), dtype=torch.uint8) if sum(map(len, hosts)) \
        else torch.zeros(0, dtype=torch.uint8)
    hrecv = torch.empty(int(r_in[:, 0].sum()), dtype=torch.uint8)
    dist.all_to_all_single(hrecv, hsend, r_in[:, 0].tolist(), s_out[:, 0].tolist(), group=ctrl_group)
    # device parts (RCCL over xGMI on MI355X: the store device's buffers as they are)
    parts = [bufs[j].to(data_dev) if bufs[j] is not None else torch.zeros(0, dtype=torch.uint8, device=data_dev)
             for j in range(k)]
    dsend = torch.cat(parts)
    drecv = torch.empty(int(r_in[:, 1].sum()), dtype=torch.uint8, device=data_dev)
    dist.all_to_all_single(drecv, dsend, r_in[:, 1].tolist(), s_out[:, 1].tolist(), group=data_group)
    got = []
    ho = do = 0
    hr = hrecv.numpy().tobytes()
    err = None
    try:
        for j in range(k):
            hn, dn = int(r_in[j, 0]), int(r_in[j, 1])
            if hn:
                b = unpack(hv, drecv[do:do + dn], hr[ho:ho + hn], verify=verify)
                if b is not None:
                    got.extend(b.ids)
            ho += hn
            do += dn
    except Exception as e:  # noqa: BLE001 - reported to every member below
        err = e
    # acknowledgement round: the move commits only if every receiver registered
    # everything it was sent; otherwise every receiver undoes what it registered and
    # every member raises, so senders keep their sessions and routes stay unchanged
    ok = torch.tensor([0 if err is not None else 1], dtype=torch.int64)
    dist.all_reduce(ok, op=dist.ReduceOp.MIN, group=ctrl_group)
    if int(ok) == 1:
        return got
    if got:
        evict(hv, got)
    if err is not None:
        raise MigrationError(f"rank {rank}: receiving migrated sessions failed: {err}") from err
    raise MigrationError(f"rank {rank}: another member failed to receive its sessions; the move was undone")


class MigrationError(RuntimeError):
    """A migration that did not commit on every member (nothing moved)."""


def all_gather_json(obj, world: int, group=None) -> list:
    """Every rank's JSON-able ``obj`` (a length all-gather, then the padded bytes)."""
    raw = json.dumps(obj).encode()
    n = torch.tensor([len(raw)], dtype=torch.int64)
    ns = [torch.zeros(1, dtype=torch.int64) for _ in range(world)]
    dist.all_gather(ns, n, group=group)
    m = max(int(x) for x in ns)
    mine = torch.zeros(m, dtype=torch.uint8)
    if raw:
        mine[:len(raw)] = torch.frombuffer(bytearray(raw), dtype=torch.uint8)
    outs = [torch.zeros(m, dtype=torch.uint8) for _ in range(world)]
    dist.all_gather(outs, mine, group=group)
    return [json.loads(o[:int(k)].numpy().tobytes().decode()) for o, k in zip(outs, ns)]


def balance_plan(loads: list, members: list) -> list:
    """Moves ``[(src, dst, count)]`` that bring every member within one session of
    the mean (the same on every rank: a pure function of the gathered loads)."""
    total = sum(loads[r] for r in members)
    k = len(members)
    target = {r: total // k + (1 if i < total % k else 0) for i, r in enumerate(members)}
    surplus = [[r, loads[r] - target[r]] for r in members if loads[r] > target[r]]
    deficit = [[r, target[r] - loads[r]] for r in members if loads[r] < target[r]]
    out = []
    i = j = 0
    while i < len(surplus) and j < len(deficit):
        c = min(surplus[i][1], deficit[j][1])
        out.append((surplus[i][0], deficit[j][0], c))
        surplus[i][1] -= c
        deficit[j][1] -= c
        if surplus[i][1] == 0:
            i += 1
        if deficit[j][1] == 0:
            j += 1
    return out


__all__ = ["pack", "unpack", "evict", "exchange", "all_gather_json", "balance_plan", "MigrationError"]
