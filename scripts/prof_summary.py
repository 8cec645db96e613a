#!/usr/bin/env python3
"""Summarise a rocprofv3 kernel-trace database (rocpd SQLite) into a markdown
table: per-kernel calls, total/mean/min/max µs, share of GPU time, and the
launch resources (VGPR/SGPR/LDS/scratch) recorded by the tracer.

    python scripts/prof_summary.py gpurun_out/prof/run_results.db > profiles/x.md
"""

from __future__ import annotations

import sqlite3
import sys


def main(path: str) -> None:
    c = sqlite3.connect(path)
    rows = c.execute(
        """select name, count(*), sum(duration), avg(duration), min(duration), max(duration),
                  max(vgpr_count), max(accum_vgpr_count), max(sgpr_count), max(lds_size),
                  max(scratch_size), max(grid_x), max(workgroup_x)
           from kernels group by name order by sum(duration) desc"""
    ).fetchall()
    total = sum(r[2] for r in rows) or 1
    print(f"source: `{path}`  (durations in µs, from rocprofv3 --kernel-trace)\n")
    print("| kernel | calls | total µs | mean µs | min µs | max µs | % GPU | VGPR | AGPR | SGPR | LDS B "
          "| scratch B | grid | wg |")
    print("|---|---|---|---|---|---|---|---|---|---|---|---|---|---|")
    for r in rows:
        name = r[0] if len(r[0]) < 90 else r[0][:87] + "..."
        print(
            f"| `{name}` | {r[1]} | {r[2]/1e3:.1f} | {r[3]/1e3:.2f} | {r[4]/1e3:.2f} | {r[5]/1e3:.2f} | "
            f"{100*r[2]/total:.1f} | {r[6]} | {r[7]} | {r[8]} | {r[9]} | {r[10]} | {r[11]} | {r[12]} |"
        )


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/prof/run_results.db")
