#!/usr/bin/env python3
"""Summarise rocprofv3 ``--pmc`` CSV output (``pmc_counter_collection.csv``) into a
markdown table: one row per kernel, each counter summed over its instances
(SE/XCD dimensions) per dispatch, then averaged over the kernel's dispatches.

    python scripts/pmc_summary.py gpurun_out/round/pmc_pipe_mix/pmc_counter_collection.csv
"""

from __future__ import annotations

import collections
import csv
import sys


def summarise(path: str) -> str:
    per_dispatch: dict = collections.defaultdict(lambda: collections.defaultdict(float))
    names = {}
    for r in csv.DictReader(open(path)):
        d = r["Dispatch_Id"]
        names[d] = r["Kernel_Name"]
        per_dispatch[d][r["Counter_Name"]] += float(r["Counter_Value"])
    by_kernel: dict = collections.defaultdict(list)
    for d, ctr in per_dispatch.items():
        by_kernel[names[d]].append(ctr)
    counters = sorted({c for ctrs in per_dispatch.values() for c in ctrs})
    out = [f"source: `{path}` (per-dispatch totals, mean over dispatches)\n",
           "| kernel | dispatches | " + " | ".join(counters) + " |",
           "|---|---|" + "---|" * len(counters)]
    for k, rows in sorted(by_kernel.items(), key=lambda kv: kv[0]):
        name = k if len(k) < 70 else k[:67] + "..."
        means = [sum(r.get(c, 0.0) for r in rows) / len(rows) for c in counters]
        out.append(f"| `{name}` | {len(rows)} | " + " | ".join(f"{m:,.0f}" for m in means) + " |")
    return "\n".join(out)


if __name__ == "__main__":
    for p in sys.argv[1:]:
        print(summarise(p))
        print()
