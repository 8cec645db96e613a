"""Audit kernels: K11/K12 batched SHA-256, K09 segmented Merkle roots, K10
non-mutating chain verification (reference audit/delta.py, session/sso.py:214,
saga/checkpoint.py:32-36)."""

from __future__ import annotations

from typing import Optional, Sequence

import torch

from agent_hypervisor_amd.ops._launch import launch

u8, i32, i64 = torch.uint8, torch.int32, torch.int64


def pack_bytes(msgs: Sequence[bytes], device="cpu") -> tuple[torch.Tensor, torch.Tensor]:
    """Byte arena + offsets[n+1] for a list of messages."""
    offs = [0]
    for m in msgs:
        offs.append(offs[-1] + len(m))
    arena = b"".join(msgs) or b"\0"
    data = torch.frombuffer(bytearray(arena), dtype=u8).to(device)
    return data, torch.tensor(offs, dtype=i64, device=device)


def digests_to_hex(d: torch.Tensor) -> list[str]:
    return ["".join(f"{w & 0xFFFFFFFF:08x}" for w in row) for row in d.cpu().tolist()]


def hex_to_digests(hexes: Sequence[str], device="cpu") -> torch.Tensor:
    rows = [[int(h[8 * k : 8 * k + 8], 16) for k in range(8)] for h in hexes]
    t = torch.tensor(rows, dtype=torch.int64).to(torch.int32) if rows else torch.zeros((0, 8), dtype=i32)
    return t.to(device)


def sha256_many(data: torch.Tensor, offsets: torch.Tensor) -> torch.Tensor:
    """SHA-256 of every message [offsets[i], offsets[i+1]) → int32 [n, 8] words."""
    n = offsets.numel() - 1
    out = torch.empty((n, 8), dtype=i32, device=data.device)
    launch("hash_many", {"n": n}, dict(bytes=data, offsets=offsets, digest=out), dict(bytes=u8, offsets=i64))
    return out


def render_rows(out: torch.Tensor, template: torch.Tensor, ids: torch.Tensor, stamps: Sequence = (),
                hex_field: Optional[tuple] = None, check: bool = True, pitch: Optional[int] = None) -> None:
    """Render audit payload rows in place: row ``ids[r]`` of ``out`` (u8, rows
    ``pitch`` bytes apart, default ``template.numel()``) becomes ``template`` with

    * each stamp ``(pos, width, mod, add)``: the decimal of ``ids[r] % mod + add``
      (``mod`` 0 = no modulus), zero-padded to ``width`` digits at ``pos``;
    * ``hex_field = (pos, src, nbytes)``: lowercase hex of the first ``nbytes``
      bytes of row ``ids[r]`` of ``src`` (any dtype, viewed as bytes) at ``pos``.

    One launch for every byte of every row (the per-session payload variation
    of re-hashed audit records, written next to the resident arena).
    ``check=False`` skips the bounds check of ``ids`` (a device sync) when the
    caller guarantees ``0 <= ids < out.numel() // len(template)`` (and the hex
    source has that many rows)."""
    L = template.numel()
    P = L if pitch is None else int(pitch)
    if P < L:
        raise ValueError("render_rows: pitch shorter than the template")
    rows = ids.numel()
    if check and rows:
        hi, lo = int(ids.max()), int(ids.min())
        limit = (out.numel() - L) // P + 1 if out.numel() >= L else 0
        if hex_field is not None:
            limit = min(limit, hex_field[1].shape[0])
        if lo < 0 or hi >= limit:
            raise ValueError(f"render_rows: row ids in [{lo}, {hi}] outside [0, {limit})")
    hp, src, nb, stride = -1, None, 0, 0
    if hex_field is not None:
        hp, hsrc, nb = hex_field
        src = hsrc.contiguous().view(torch.uint8).reshape(hsrc.shape[0], -1)
        stride = src.shape[1]
        if nb > stride:
            raise ValueError("hex field longer than its source rows")
    launch("render_rows",
           {"rows": rows, "len": L, "pitch": P, "stamps": [tuple(int(x) for x in st) for st in stamps],
            "hex_pos": int(hp),
            "hex_bytes": int(nb), "hex_stride": int(stride)},
           dict(tmpl=template, out=out, ids=ids, hex_src=src), dict(tmpl=u8, out=u8, ids=i64, hex_src=u8))


def content_hashes(contents: Sequence[str], device="cpu") -> list[str]:
    """K11: sha256(content.encode()).hexdigest() for many VFS contents."""
    data, offs = pack_bytes([c.encode() for c in contents], device)
    return digests_to_hex(sha256_many(data, offs))


def goal_hashes(goals: Sequence[str], step_ids: Sequence[str], device="cpu") -> list[str]:
    """K12: SemanticCheckpoint.compute_goal_hash for many (goal, step) pairs."""
    data, offs = pack_bytes([f"{g}:{s}".encode() for g, s in zip(goals, step_ids)], device)
    return [h[:16] for h in digests_to_hex(sha256_many(data, offs))]


def merkle_roots(offsets: torch.Tensor, leaves: torch.Tensor, leaf_idx: Optional[torch.Tensor] = None,
                 root_out: Optional[torch.Tensor] = None, root_row: Optional[torch.Tensor] = None,
                 gate: Optional[torch.Tensor] = None) -> torch.Tensor:
    """K09: Merkle root of each chain of leaf digests (zeros for empty chains).

    Fused forms: ``leaf_idx`` (int64) — leaf i of the concatenated chains is row
    ``leaf_idx[i]`` of ``leaves`` (a resident digest table: no gathered copy);
    ``root_out`` + ``root_row`` (int64) — root c is written to row ``root_row[c]``
    of ``root_out`` (e.g. the store's ``s_root``), zeros where ``gate[row] == 0``."""
    chains = offsets.numel() - 1
    nleaf = leaf_idx.numel() if leaf_idx is not None else leaves.shape[0]
    root = root_out if root_out is not None else torch.empty((chains, 8), dtype=i32, device=leaves.device)
    scratch = torch.empty((max(1, nleaf), 8), dtype=i32, device=leaves.device)
    tensors = dict(offsets=offsets, leaves=leaves, scratch=scratch, root=root)
    dtypes = dict(offsets=i32, leaves=i32)
    if leaf_idx is not None:
        if offsets.device.type == "cpu" and nleaf and int(leaf_idx.max()) >= leaves.shape[0]:
            raise IndexError("merkle_roots: leaf_idx out of range")
        tensors["leaf_idx"], dtypes["leaf_idx"] = leaf_idx, torch.int64
    if root_row is not None:
        if root_out is None:
            raise ValueError("merkle_roots: root_row needs root_out")
        tensors["root_row"], dtypes["root_row"] = root_row, torch.int64
        if gate is not None:
            tensors["gate"], dtypes["gate"] = gate, torch.int64
    launch("merkle", {"chains": chains}, tensors, dtypes)
    return root


def merkle_tree_root(leaves: torch.Tensor) -> torch.Tensor:
    """K09 work-parallel: Merkle root ([8] int32) of ONE chain of ``n`` leaf digests.

    Multi-pass over ``csrc/hip/merkle_tree.hip``: each pass reduces
    L = min(9, ⌈log2 count⌉) levels with one 256-thread workgroup per aligned
    2^L-leaf subtree (LDS-resident levels), until one node is left.  Exactly the
    reference tree (odd duplication, a single leaf is its own root)."""
    if leaves.dim() != 2 or leaves.shape[1] != 8 or leaves.dtype != torch.int32:
        raise TypeError("leaves must be an int32 [n, 8] digest tensor")
    n = leaves.shape[0]
    if n == 0:
        raise ValueError("no leaves")
    cur = leaves.contiguous()
    while cur.shape[0] > 1:
        count = cur.shape[0]
        levels = min(9, (count - 1).bit_length())
        out = torch.empty(((count + (1 << levels) - 1) >> levels, 8), dtype=torch.int32, device=cur.device)
        launch("merkle_tree_pass", {"count": count, "levels": levels}, {"in": cur, "out": out})
        cur = out
    return cur[0]


def verify_chains(
    data: torch.Tensor,
    offsets: torch.Tensor,
    stored: torch.Tensor,
    parent: torch.Tensor,
    has_parent: torch.Tensor,
    chain_offsets: torch.Tensor,
) -> tuple[torch.Tensor, torch.Tensor]:
    """K10: per-delta and per-chain integrity of canonical payloads vs stored
    digests and parent links → (delta_ok u8 [D], chain_ok u8 [C])."""
    D = offsets.numel() - 1
    Cn = chain_offsets.numel() - 1
    dok = torch.empty(D, dtype=u8, device=data.device)
    cok = torch.empty(Cn, dtype=u8, device=data.device)
    launch(
        "verify",
        {"deltas": D, "chains": Cn},
        dict(bytes=data, offsets=offsets, stored=stored, parent=parent, has_parent=has_parent,
             chain_offsets=chain_offsets, delta_ok=dok, chain_ok=cok),
        dict(bytes=u8, offsets=i64, stored=i32, parent=i32, has_parent=u8, chain_offsets=i32),
    )
    return dok, cok


_PARENT_MARK = "@@ahv-parent-field@@"


def _split_payload(d) -> tuple[bytes, bytes]:
    """Canonical payload of ``d`` split around its parent_hash value."""
    import dataclasses

    from hypervisor.audit.delta import canonical_payload

    marked = dataclasses.replace(d, parent_hash=_PARENT_MARK)
    text = canonical_payload(marked).decode("ascii")
    import json

    pieces = text.split(json.dumps(_PARENT_MARK))
    if len(pieces) != 2:
        raise ValueError(f"delta {d.delta_id} contains the parent placeholder text")
    return pieces[0].encode(), pieces[1].encode()


def pack_chains(chains, device="cpu") -> dict:
    """Pack lists of SemanticDelta (one list per chain) for :func:`chain_hashes`:
    each payload is stored as (prefix, suffix) around the parent field."""
    parts, pre_off, pre_len, suf_off, suf_len, offs = [], [], [], [], [], [0]
    pos = 0
    for chain in chains:
        for d in chain:
            pre, suf = _split_payload(d)
            pre_off.append(pos)
            pre_len.append(len(pre))
            parts.append(pre)
            pos += len(pre)
            suf_off.append(pos)
            suf_len.append(len(suf))
            parts.append(suf)
            pos += len(suf)
        offs.append(len(pre_off))
    arena = b"".join(parts) or b"\0"
    t = lambda xs, dt: torch.tensor(xs, dtype=dt, device=device)  # noqa: E731
    return dict(
        bytes=torch.frombuffer(bytearray(arena), dtype=u8).to(device),
        chain_offsets=t(offs, i32), pre_off=t(pre_off, i64), pre_len=t(pre_len, i32),
        suf_off=t(suf_off, i64), suf_len=t(suf_len, i32),
    )


def chain_hashes(packed: dict, seed_parent: Optional[torch.Tensor] = None,
                 has_seed: Optional[torch.Tensor] = None, midstate: bool = True,
                 uniform_len: int = 0, sel: Optional[torch.Tensor] = None, check: bool = True) -> torch.Tensor:
    """K08: re-derive every delta hash of every chain (parent links recomputed
    from the chain itself) → int32 [D, 8].

    ``midstate=True`` splits the work in two launches: every delta's whole
    prefix blocks (the chain-independent bytes before ``"parent_hash"``) are
    compressed in parallel, one lane per delta; the serial per-chain pass then
    resumes from those midstates.

    ``uniform_len`` (> 0) promises that every chain holds exactly that many
    deltas; phase 1 then assigns a wave the same turn of 64 chains (payloads of
    one shape) instead of consecutive deltas of a few chains.

    ``sel`` (int64 [chains], with ``uniform_len``) reads chain c's spans from
    rows ``sel[c]·len …`` of the span tables in ``packed`` — resident
    per-session tables — instead of gathering them per call; ``chain_offsets``
    must then be the uniform ``c·len``.  Digests come back in chain order.
    ``check=False`` skips the range check of ``sel`` (a device sync) when the
    caller guarantees every row exists."""
    dev = packed["bytes"].device
    chains = packed["chain_offsets"].numel() - 1
    if sel is not None:
        if uniform_len <= 0 or sel.numel() != chains:
            raise ValueError("sel needs uniform_len and one row per chain")
        rows = min(packed[k].numel() for k in ("pre_off", "pre_len", "suf_off", "suf_len")) // uniform_len
        if check and chains and not (0 <= int(sel.min()) and int(sel.max()) < rows):
            raise ValueError(f"sel rows outside the span tables' {rows} rows")
        D = chains * uniform_len
    else:
        D = packed["pre_off"].numel()
    if uniform_len and (uniform_len < 0 or chains * uniform_len != D):
        raise ValueError(f"uniform_len={uniform_len} does not match {chains} chains of {D} deltas")
    out = torch.empty((D, 8), dtype=i32, device=dev)
    mid = torch.empty((D, 8), dtype=i32, device=dev) if midstate and D else None
    launch(
        "chain_hash",
        {"chains": packed["chain_offsets"].numel() - 1, "deltas": D, "uniform_len": int(uniform_len)},
        dict(packed, seed_parent=seed_parent, has_seed=has_seed, digest=out, mid=mid, sel=sel),
        dict(bytes=u8, chain_offsets=i32, pre_off=i64, pre_len=i32, suf_off=i64, suf_len=i32,
             seed_parent=i32, has_seed=u8, mid=i32, sel=i64),
    )
    return out


def pack_delta_engines(engines, device="cpu"):
    """Pack DeltaEngine chains for :func:`verify_chains` / :func:`merkle_roots`."""
    from hypervisor.audit.delta import canonical_payload

    payloads, stored, parent, has_parent, chain_offs = [], [], [], [], [0]
    for de in engines:
        for d in de.deltas:
            payloads.append(canonical_payload(d))
            stored.append(d.delta_hash if len(d.delta_hash) == 64 else "0" * 64)
            parent.append(d.parent_hash if d.parent_hash and len(d.parent_hash) == 64 else "0" * 64)
            has_parent.append(1 if d.parent_hash is not None else 0)
        chain_offs.append(len(payloads))
    data, offs = pack_bytes(payloads, device)
    return (
        data,
        offs,
        hex_to_digests(stored, device),
        hex_to_digests(parent, device),
        torch.tensor(has_parent, dtype=u8, device=device),
        torch.tensor(chain_offs, dtype=i32, device=device),
    )
