#!/usr/bin/env python3
"""Phase timeline of the cooperative small-batch template kernel
(``store_template_coop_kernel``, csrc/hip/store_template.hip): per wave of
workgroup 0, the s_memrealtime stamps (10 ns) the kernel writes at its phase
boundaries when handed a ``phase_ticks`` buffer, in µs from the kernel's first
stamp; median over launches.  ``python scripts/coop_phases.py [sessions]``."""
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from agent_hypervisor_amd.models import store_template as TT  # noqa: E402
from agent_hypervisor_amd.models.store import GovernanceStore  # noqa: E402

NAMES = {
    0: ["start", "render", "-", "chain r0", "published", "n01+root blk1"],
    1: ["start", "render", "prefix r1", "chain r1", "published", "root"],
    2: ["start", "render", "prefix r2", "chain r2", "published"],
    3: ["start", "session rows", "schedules produced", "events"],
}


def main() -> None:
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000
    st = GovernanceStore("cuda", caps={"S": 2 * n, "G": 2 * n, "T": 2 * n, "D": 8 * n, "B": 8 * n * 512})
    agents = TT.AgentSet.synthetic(st, 2048, seed=3, prefix="did:mesh:agent-")
    tp = TT.TemplatePipeline(st, n, agents, deltas=3)
    ticks = torch.zeros(64, dtype=torch.int64, device="cuda")
    rows = []
    for k in range(30):
        sa = torch.randint(0, agents.count, (n,), dtype=torch.int32, device="cuda")
        ticks.zero_()
        tp.reset()
        tp.launch(sa, sync=True, extra={"phase_ticks": ticks.data_ptr()})
        rows.append(ticks.view(4, 16).cpu().numpy().copy())
    out = {}
    for w in range(4):
        base = [r[0, 0] for r in rows[5:]]
        for k, name in enumerate(NAMES[w]):
            if name == "-":
                continue
            v = [(r[w, k] - b) / 100.0 for r, b in zip(rows[5:], base) if r[w, k]]
            if v:
                out[f"w{w}.{k}.{name}"] = round(statistics.median(v), 2)
    print(json.dumps({"sessions": n, "kernel": "store_template_coop_kernel", "us_from_start": out}, indent=1))


if __name__ == "__main__":
    main()
