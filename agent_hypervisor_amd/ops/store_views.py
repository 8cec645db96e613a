"""Batched reductions over the device store's resident tables (one device state).

The public API's state lives in :class:`agent_hypervisor_amd.models.store.GovernanceStore`
columns; these views reduce those columns directly on the device — no per-row
command, no host copy of the rows — for the agent-global views of the sharded
hypervisor (X01) and the batched audit/liability paths.
"""

from __future__ import annotations

import torch

from hypervisor._clock import now_us


def exposure_by_agent(store, agent_ids: list[int], edges: list[int], now: int | None = None) -> torch.Tensor:
    """K04 over store edges: Σ bonded amount of the *live* edges (active, not expired
    at ``now``) among ``edges``, per voucher, for the agents ``agent_ids`` (store
    agent ids, −1 = unknown agent → 0), as fp64 [len(agent_ids)] on the store device."""
    dev = store.device
    n = len(agent_ids)
    out = torch.zeros(n, dtype=torch.float64, device=dev)
    if not edges or not n:
        return out
    t = int(now if now is not None else now_us())
    e = torch.as_tensor(edges, dtype=torch.int64).to(dev)
    voucher = store.column("e_voucher").index_select(0, e).to(torch.int64)
    bonded = store.tables["e_bonded"].index_select(0, e)
    active = store.tables["e_active"].index_select(0, e).bool()
    expiry = store.tables["e_expiry"].index_select(0, e)
    live = active & ((expiry < 0) | (expiry >= t))
    ids = torch.as_tensor(agent_ids, dtype=torch.int64).to(dev)
    known = ids >= 0
    space = int(max(int(voucher.max()) if voucher.numel() else 0, int(ids.max()) if n else 0)) + 1
    lut = torch.full((space,), -1, dtype=torch.int64, device=dev)
    lut[ids[known]] = torch.arange(n, device=dev)[known]
    slot = lut[voucher.clamp(min=0)]
    keep = live & (slot >= 0) & (voucher >= 0)
    out.index_add_(0, slot[keep], bonded[keep])
    return out
