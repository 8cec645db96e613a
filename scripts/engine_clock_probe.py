"""Is the lone hash-engine wave slow because the GPU clocks down when one CU is busy?
Runs scripts/engine_probe.py's measurement twice: idle GPU, then with a background
stream keeping the other CUs busy (bf16 GEMMs).  Evidence only — not a runtime mode."""
import asyncio
import json
import sys
import threading

import torch

sys.path.insert(0, "scripts")
sys.path.insert(0, ".")
import engine_probe  # noqa: E402

idle = asyncio.run(engine_probe.main(300))
stop = threading.Event()


def heater():
    s = torch.cuda.Stream()
    a = torch.randn(4096, 4096, device="cuda", dtype=torch.bfloat16)
    with torch.cuda.stream(s):
        while not stop.is_set():
            for _ in range(8):
                a = (a @ a).clamp_(-1, 1)
            s.synchronize()


t = threading.Thread(target=heater, daemon=True)
t.start()
busy = asyncio.run(engine_probe.main(300))
stop.set()
t.join()
print(json.dumps({"idle": idle, "busy_gpu": busy}), flush=True)
