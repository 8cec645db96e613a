"""Where the batched heterogeneous API's host time goes: cProfile of prepare() and
finish() over 2·10⁴ random specs (the bench_api hetero batch), after a warm-up."""
import cProfile
import os
import pstats
import random
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from test_store_pipeline import random_spec  # noqa: E402

from hypervisor import Hypervisor  # noqa: E402
from agent_hypervisor_amd.models import store_pipeline as SP  # noqa: E402
from agent_hypervisor_amd._native import C  # noqa: E402

dev = sys.argv[1] if len(sys.argv) > 1 else "cuda"
rng = random.Random(5)
specs = [random_spec(rng) for _ in range(20000)]
hv = Hypervisor(device=dev)
st = hv._store
for _ in range(2):
    p = SP.prepare(hv, specs)
    SP.launch(p)
    r = SP.finish(hv, p)
for th in (1, 2, 4, 8, 16, -1):
    ts = []
    for _ in range(3):
        t = time.perf_counter()
        C.pack_specs(specs, st.agents._pool, st.pool._pool, lambda c: (4, 0.5, 1), SP._FIXED, th)
        ts.append(time.perf_counter() - t)
    print("pack_specs threads", th, "ms", [round(x * 1e3, 2) for x in ts], flush=True)
pr = cProfile.Profile()
pr.enable()
p = SP.prepare(hv, specs)
SP.launch(p)
r = SP.finish(hv, p)
pr.disable()
pstats.Stats(pr).sort_stats("tottime").print_stats(18)
