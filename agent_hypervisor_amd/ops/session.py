"""Session-concurrency kernels: K19 vector clocks, K20 intent-lock contention
(reference session/vector_clock.py:71-165, session/intent_locks.py:158-178)."""

from __future__ import annotations

import torch

from agent_hypervisor_amd.ops._launch import launch

u8, i32 = torch.uint8, torch.int32
READ, WRITE = 0, 1
LOCK_INTENT = {"read": 0, "write": 1, "exclusive": 2}


def vector_clock_ops(offsets, op, path, agent, agent_col, path_clock, agent_clock, strict=True) -> torch.Tensor:
    """Apply read/write ops (grouped, in order) to dense clocks in place → ok u8.

    ``path_clock`` / ``agent_clock`` are int32 [rows, A] with A ≤ 64 components."""
    ok = torch.empty(op.numel(), dtype=u8, device=op.device)
    launch(
        "vclock",
        {"groups": offsets.numel() - 1, "A": path_clock.shape[1], "strict": int(bool(strict))},
        dict(offsets=offsets, op=op, path=path, agent=agent, agent_col=agent_col, path_clock=path_clock,
             agent_clock=agent_clock, ok=ok),
        dict(offsets=i32, op=u8, path=i32, agent=i32, agent_col=i32, path_clock=i32, agent_clock=i32),
    )
    return ok


def lock_conflicts(res_offsets, lock_agent, lock_intent, req_res, req_agent, req_intent) -> torch.Tensor:
    """Number of active locks each request conflicts with (0 = grantable)."""
    out = torch.empty(req_res.numel(), dtype=i32, device=req_res.device)
    launch(
        "locks",
        {"n": req_res.numel()},
        dict(res_offsets=res_offsets, lock_agent=lock_agent, lock_intent=lock_intent, req_res=req_res,
             req_agent=req_agent, req_intent=req_intent, conflicts=out),
        dict(res_offsets=i32, lock_agent=i32, lock_intent=u8, req_res=i32, req_agent=i32, req_intent=u8),
    )
    return out


LOCK_HOLDERS = 16
LOCK_ROW = 2 + 2 * LOCK_HOLDERS
LOCK_RELEASE = 0x80


def lock_grant(seg_offsets, order, req_res, req_agent, req_intent, table, granted) -> None:
    """K20 grant pass over the resident holder tables ``table`` [R, LOCK_ROW]
    (in place); see ``LockGrantArgs`` in csrc/include/ahv/kernels.h."""
    if table.dim() != 2 or table.shape[1] != LOCK_ROW or not table.is_contiguous():
        raise ValueError(f"lock table must be contiguous int32 [R, {LOCK_ROW}]")
    launch(
        "lock_grant",
        {"segments": seg_offsets.numel() - 1},
        dict(seg_offsets=seg_offsets, order=order, req_res=req_res, req_agent=req_agent, req_intent=req_intent,
             table=table, granted=granted),
        dict(seg_offsets=i32, order=i32, req_res=i32, req_agent=i32, req_intent=u8, table=i32, granted=u8),
    )
