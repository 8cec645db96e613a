#!/usr/bin/env python3
"""Summarise rocprofv3 ``--pmc`` output (``pmc_counter_collection.csv`` or the rocpd
``*_results.db``) into a
markdown table: one row per kernel, each counter summed over its instances
(SE/XCD dimensions) per dispatch, then averaged over the kernel's dispatches.

    python scripts/pmc_summary.py gpurun_out/round/pmc_pipe_mix/pmc_counter_collection.csv
"""

from __future__ import annotations

import collections
import csv
import sys


def _rows(path: str):
    """(dispatch id, kernel name, counter, value) from the CSV or the rocpd SQLite database."""
    if path.endswith(".db"):
        import sqlite3

        c = sqlite3.connect(path)
        yield from c.execute("select dispatch_id, kernel_name, counter_name, value from counters_collection")
        return
    for r in csv.DictReader(open(path)):
        yield r["Dispatch_Id"], r["Kernel_Name"], r["Counter_Name"], r["Counter_Value"]


def summarise(path: str) -> str:
    per_dispatch: dict = collections.defaultdict(lambda: collections.defaultdict(float))
    names = {}
    for d, k, cn, v in _rows(path):
        names[d] = k
        per_dispatch[d][cn] += float(v)
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
