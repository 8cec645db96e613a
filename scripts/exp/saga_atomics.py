"""Experiment: cost of same-address counter atomics in the fused saga kernel."""
import time, torch
from agent_hypervisor_amd._native import C
from agent_hypervisor_amd.models.saga_engine import SagaBatchEngine, SagaOutcomes

S, K = 1_000_000, 10
dev = torch.device("cuda", 0)
o = SagaOutcomes.synthetic(S, K, p_fail=0.03, p_comp_fail=0.05, p_no_undo=0.05, max_retries=1).to(dev)
e = SagaBatchEngine(S, K, device="cuda")
a = e._args(o, 1)
st = torch.cuda.current_stream(dev).cuda_stream
for label, args in (("with stats", a), ("no stats", dict(a, stats=None))):
    for _ in range(3):
        C.saga_fused(args, st)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(20):
        C.saga_fused(args, st)
    torch.cuda.synchronize()
    print(label, (time.perf_counter() - t0) / 20 * 1e3, "ms")
# python-side overhead of run()
torch.cuda.synchronize(); t0 = time.perf_counter()
for _ in range(20):
    e.run(o, now_us=1)
torch.cuda.synchronize(); print("engine.run", (time.perf_counter() - t0) / 20 * 1e3, "ms")
