"""cProfile of execute_sagas(device=...) with 4096 stub-coroutine sagas x 10 steps
(config4 coroutine mode) against the host orchestrator."""
import asyncio
import cProfile
import pstats
import random
import sys
import time

sys.path.insert(0, ".")
from hypervisor.saga.orchestrator import SagaOrchestrator  # noqa: E402

K, S = 10, 4096
DEV = sys.argv[1] if len(sys.argv) > 1 else "cuda"


def build(seed=0):
    rng = random.Random(seed)
    orch = SagaOrchestrator()
    orch.DEFAULT_RETRY_DELAY_SECONDS = 0.0
    ids, ex = [], {}
    for i in range(S):
        sg = orch.create_saga(f"session-{i}")
        ids.append(sg.saga_id)
        for k in range(K):
            st = orch.add_step(sg.saga_id, f"a{k}", "did:mesh:agent", "/exec",
                               "/undo" if rng.random() >= 0.05 else None, max_retries=1)
            fail = rng.random() < 0.03

            async def run(fail=fail):
                if fail:
                    raise RuntimeError("executor failed")
                return True

            ex[st.step_id] = run
    return orch, ids, ex


async def comp(step):
    return True


for dev in (None, DEV, None, DEV, None, DEV):
    orch, ids, ex = build()
    t0 = time.perf_counter()
    asyncio.run(orch.execute_sagas(ids, ex, comp, device=dev))
    print(dev, round((time.perf_counter() - t0) * 1e3, 1), "ms", flush=True)
orch, ids, ex = build()
pr = cProfile.Profile()
pr.enable()
asyncio.run(orch.execute_sagas(ids, ex, comp, device=DEV))
pr.disable()
pstats.Stats(pr).sort_stats("tottime").print_stats(18)
