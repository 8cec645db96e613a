"""Per-call API under asyncio.gather on the device store: throughput and a cProfile
of one 2,000-pipeline batch (where the Python time goes)."""
import asyncio
import cProfile
import gc
import io
import json
import pstats
import sys

sys.path.insert(0, ".")
sys.path.insert(0, "benchmarks")
from bench_api import api_throughput, reference_pipeline  # noqa: E402

dev = sys.argv[1] if len(sys.argv) > 1 else "cuda"
import time  # noqa: E402

from agent_hypervisor_amd.models.store import shared_store  # noqa: E402

st = shared_store(dev)
i0, t0 = st.info(), time.perf_counter()
res = api_throughput(dev, 10_000, rounds=3)
i1, wall = st.info(), time.perf_counter() - t0
if "worker_busy_us" in i1:  # store worker utilisation over the whole measurement (warm-up included)
    res["worker_busy_frac"] = round((i1["worker_busy_us"] - i0["worker_busy_us"]) / (wall * 1e6), 4)
    res["engine_busy_frac"] = round((i1["engine_busy_us"] - i0["engine_busy_us"]) / (wall * 1e6), 4)
    res["commands"] = i1["worker_commands"] - i0["worker_commands"]
    res["us_per_command_busy"] = round((i1["worker_busy_us"] - i0["worker_busy_us"]) / max(1, res["commands"]), 3)
    res["wall_s"] = round(wall, 3)
print(json.dumps(res), flush=True)
print(json.dumps(api_throughput("host", 10_000, rounds=3)), flush=True)


async def batch(k):
    return await asyncio.gather(*[reference_pipeline(dev) for _ in range(k)])


from hypervisor.config import tune_gc  # noqa: E402

tune_gc()
asyncio.run(batch(500))
gc.collect()
pr = cProfile.Profile()
pr.enable()
asyncio.run(batch(2000))
pr.disable()
s = io.StringIO()
pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(30)
print(s.getvalue())
