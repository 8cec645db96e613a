"""Where the host time of Hypervisor.run_pipelines goes (10^5 template pipelines)."""
import asyncio
import cProfile
import gc
import io
import pstats
import sys
import time

sys.path.insert(0, ".")
from agent_hypervisor_amd.models.store_pipeline import PipelineSpec  # noqa: E402
from hypervisor import Hypervisor  # noqa: E402

n = 100_000


async def one():
    hv = Hypervisor(device="cuda")
    r = await hv.run_pipelines(PipelineSpec(), n)
    return hv, r


hv, r = asyncio.run(one())
del hv, r
gc.collect()
for _ in range(2):
    t0 = time.perf_counter()
    hv, r = asyncio.run(one())
    t1 = time.perf_counter()
    del hv, r
    t2 = time.perf_counter()
    print(f"run {1e3 * (t1 - t0):.1f} ms  teardown {1e3 * (t2 - t1):.1f} ms", flush=True)
pr = cProfile.Profile()
pr.enable()
hv, r = asyncio.run(one())
del hv, r
pr.disable()
s = io.StringIO()
pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(25)
print(s.getvalue())
