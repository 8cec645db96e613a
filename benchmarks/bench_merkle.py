#!/usr/bin/env python3
"""K09 on one long chain: work-parallel tree (LDS subtrees, multi-pass) vs the
round-1 one-lane-per-chain kernel, on one MI355X.  Prints one JSON line per n."""
import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from agent_hypervisor_amd.ops.audit import merkle_roots, merkle_tree_root  # noqa: E402


def timed(fn, reps):
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b))
    return statistics.median(ts)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", default="10000,100000,1000000,10000000,16000000")
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--single-lane-max", type=int, default=100000)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    for n in (int(x) for x in args.sizes.split(",")):
        lv = torch.randint(-(2**31), 2**31 - 1, (n, 8), dtype=torch.int32, device=dev)
        merkle_tree_root(lv)
        torch.cuda.synchronize()
        t_tree = timed(lambda: merkle_tree_root(lv), args.reps)
        row = {"n_leaves": n, "tree_ms": round(t_tree, 4), "nodes_per_s": round((n - 1) / (t_tree / 1e3), 1)}
        if n <= args.single_lane_max:
            off = torch.tensor([0, n], dtype=torch.int32, device=dev)
            merkle_roots(off, lv)
            t1 = timed(lambda: merkle_roots(off, lv), max(1, args.reps // 2))
            row["single_lane_ms"] = round(t1, 4)
            row["speedup"] = round(t1 / t_tree, 1)
            assert torch.equal(merkle_roots(off, lv)[0], merkle_tree_root(lv))
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
