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
print(json.dumps(api_throughput(dev, 10_000, rounds=3)), flush=True)
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
