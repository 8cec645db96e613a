"""Saga kernels: K13 step/saga FSM, K14 compensation planning, K15 fan-out
policy (reference saga/state_machine.py, saga/orchestrator.py:145-198,
saga/fan_out.py:62-70)."""

from __future__ import annotations

import torch

from agent_hypervisor_amd.ops._launch import launch

u8, i32, i64 = torch.uint8, torch.int32, torch.int64

STEP = {"pending": 0, "executing": 1, "committed": 2, "compensating": 3, "compensated": 4,
        "compensation_failed": 5, "failed": 6}
SAGA = {"running": 0, "compensating": 1, "completed": 2, "failed": 3, "escalated": 4}
POLICY = {"all_must_succeed": 0, "majority_must_succeed": 1, "any_must_succeed": 2}


def transition(state: torch.Tensor, target: torch.Tensor, now_us: int, saga: bool = False,
               started_us=None, completed_us=None) -> torch.Tensor:
    """Apply FSM transitions in place where valid; returns ok u8 per element."""
    ok = torch.empty(state.numel(), dtype=u8, device=state.device)
    launch(
        "fsm",
        {"n": state.numel(), "kind": 1 if saga else 0, "now_us": int(now_us)},
        dict(state=state, target=target, ok=ok, started_us=started_us, completed_us=completed_us),
        dict(state=u8, target=u8, started_us=i64, completed_us=i64),
    )
    return ok


def fanout_policy(offsets: torch.Tensor, policy: torch.Tensor, succeeded: torch.Tensor):
    """(satisfied u8 [G], success_count i32 [G], compensate u8 [B])."""
    G = offsets.numel() - 1
    sat = torch.empty(G, dtype=u8, device=offsets.device)
    cnt = torch.empty(G, dtype=i32, device=offsets.device)
    comp = torch.empty(succeeded.numel(), dtype=u8, device=offsets.device)
    launch(
        "fanout",
        {"groups": G},
        dict(offsets=offsets, policy=policy, succeeded=succeeded, satisfied=sat, success_count=cnt, compensate=comp),
        dict(offsets=i32, policy=u8, succeeded=u8),
    )
    return sat, cnt, comp


def compensation_plan(step_state: torch.Tensor, has_undo: torch.Tensor, now_us: int):
    """K14 for [S, K] step tables: committed steps in reverse order are the
    compensation plan; steps without an Undo_API fail compensation.

    Returns (order i64 [S, K] of step indices to compensate, reverse order, -1
    padded; and, applied in place, COMPENSATING for compensable steps and
    COMPENSATION_FAILED for committed steps with no Undo_API)."""
    S, K = step_state.shape
    committed = step_state == STEP["committed"]
    idx = torch.arange(K, device=step_state.device).expand(S, K)
    key = torch.where(committed, idx, torch.full_like(idx, -1))
    order = torch.sort(key, dim=1, descending=True).values
    target = torch.where(has_undo.bool(), torch.full_like(step_state, STEP["compensating"]),
                         torch.full_like(step_state, STEP["compensation_failed"]))
    flat_state = step_state.reshape(-1)
    flat_target = torch.where(committed, target, step_state).reshape(-1).contiguous()
    no_undo = committed & ~has_undo.bool()
    # COMMITTED → COMPENSATION_FAILED is outside the FSM (the reference assigns it
    # directly, orchestrator.py:167-170); apply it before the FSM pass.
    flat_state[no_undo.reshape(-1)] = STEP["compensation_failed"]
    transition(flat_state, flat_target, now_us)
    return order
