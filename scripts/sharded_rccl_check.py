"""Sharded Hypervisor under torch.distributed with the RCCL ("nccl") backend and
the device store: run the mixed route scenario of tests/test_sharded.py on every
rank and check rank 0's answers against a single-rank façade.  Launched by
torch.distributed.run (tests/test_gpu_dist.py runs it with one rank)."""
import asyncio
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def main() -> None:
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    from agent_hypervisor_amd.parallel.sharded import ShardedHypervisor
    from tests.test_sharded import scenario

    async def run():
        shv = await ShardedHypervisor(device="cuda", policy="round_robin").start()
        if dist.get_rank() != 0:
            await shv.serve_forever()
            return None
        got = await scenario(shv)
        x = await shv.exposure_vector([f"did:agent-{a}" for a in range(5)])  # X01: K04 over store edges + RCCL
        counters = dict(shv.counters)
        await shv.shutdown()
        ref = await scenario(await ShardedHypervisor(device="cuda", single=True).start())
        return got, ref, x, counters, shv.local._store.is_gpu

    res = asyncio.run(run())
    ok = True
    if dist.get_rank() == 0:
        got, ref, x, counters, gpu = res
        bad = [k for k in ref if got[k] != ref[k]]
        ok = not bad
        print(json.dumps({"ok": ok, "mismatch": bad, "world": dist.get_world_size(),
                          "backend": dist.get_backend(), "exposure": x, "counters": counters,
                          "store_gpu": gpu}), flush=True)
    dist.destroy_process_group()
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
