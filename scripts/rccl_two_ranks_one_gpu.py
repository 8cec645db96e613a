#!/usr/bin/env python3
"""RCCL at world = 2 on ONE GPU: both ranks bind cuda:0 (a one-GPU box is all the
development pool offers; the driver's 8-GPU run is the real scaling test).

Exercises the C++ communicator (``parallel/rccl.py`` Communicator: all_reduce,
all_gather, reduce_scatter, broadcast, all_to_all) and the torch.distributed
"nccl" (= RCCL) process group, checking every result against its closed form.
RCCL may refuse two ranks on one device ("duplicate GPU"): then the script
prints what it reported and exits 3, which says nothing about the code.

    python -m torch.distributed.run --nnodes 1 --nproc-per-node 2 \\
        --master-addr 127.0.0.1 --master-port 29533 scripts/rccl_two_ranks_one_gpu.py
"""

from __future__ import annotations

import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main() -> int:
    import torch
    import torch.distributed as dist

    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from agent_hypervisor_amd.parallel.rccl import Communicator

    dev = torch.device("cuda", 0)
    out = {"rank": rank, "world": world}
    try:
        comm = Communicator.from_process_group(device=0)
    except Exception as e:  # noqa: BLE001 - reported, not a code failure
        out["communicator"] = f"refused: {e}"
        print(json.dumps(out), flush=True)
        return 3
    s = torch.cuda.Stream(dev)
    with torch.cuda.stream(s):
        a = torch.full((1 << 20,), float(rank + 1), dtype=torch.float32, device=dev)
        comm.all_reduce(a, stream=s)
        g = comm.all_gather(torch.full((4,), rank, dtype=torch.int64, device=dev), stream=s)
        rs = comm.reduce_scatter(torch.arange(8 * world, dtype=torch.float64, device=dev), stream=s)
        b = torch.full((16,), 7 if rank == 0 else -1, dtype=torch.int32, device=dev)
        comm.broadcast(b, root=0, stream=s)
        x = (torch.arange(4 * world, dtype=torch.int32, device=dev) + 100 * rank)
        y = comm.all_to_all(x, stream=s)
    s.synchronize()
    tot = world * (world + 1) / 2
    checks = {
        "all_reduce": bool(torch.all(a == tot)),
        "all_gather": g.cpu().tolist() == [[r] * 4 for r in range(world)],
        "reduce_scatter": torch.equal(rs.cpu(), (torch.arange(8 * world,
                                                              dtype=torch.float64) * world)[8 * rank:8 * rank + 8]),
        "broadcast": bool(torch.all(b == 7)),
        # block r of rank q's input (4 ints) lands in block q of rank r's output
        "all_to_all": y.cpu().tolist() == [v for q in range(world) for v in range(4 * rank + 100 * q,
                                                                                  4 * rank + 4 + 100 * q)],
    }
    out["rccl_version"] = Communicator.version()
    out["communicator"] = checks
    comm.destroy()
    # the torch.distributed "nccl" (RCCL) backend on the same device
    try:
        pg = dist.new_group(backend="nccl")
        t = torch.full((1024,), float(rank), device=dev)
        dist.all_reduce(t, group=pg)
        torch.cuda.synchronize(dev)
        out["torch_nccl_all_reduce"] = bool(torch.all(t == world * (world - 1) / 2))
    except Exception as e:  # noqa: BLE001
        out["torch_nccl_all_reduce"] = f"refused: {e}"
    print(json.dumps(out), flush=True)
    dist.barrier()
    dist.destroy_process_group()
    return 0 if all(checks.values()) else 1


if __name__ == "__main__":
    sys.exit(main())
