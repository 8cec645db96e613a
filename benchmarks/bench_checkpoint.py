"""Columnar checkpoint of a device-backed hypervisor at scale.

``python benchmarks/bench_checkpoint.py --sessions 1000000 --device cpu``: one
``Hypervisor.run_pipelines`` batch of reference pipelines (create → join →
activate → 3 audit deltas → saga step → terminate) into the store, then
``save_hypervisor`` (timed; store commands counted) and ``load_hypervisor`` into
a fresh hypervisor on a fresh store (timed, full K10/K09 re-verification), and
a spot check that restored sessions answer the API.  Prints one JSON line.
"""

from __future__ import annotations

import argparse
import asyncio
import json
import os
import shutil
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--sessions", type=int, default=100_000)
    ap.add_argument("--device", default="cpu")
    ap.add_argument("--dir", default=None)
    args = ap.parse_args()

    from agent_hypervisor_amd.models.store import GovernanceStore
    from agent_hypervisor_amd.models.store_pipeline import PipelineSpec
    from agent_hypervisor_amd.runtime.checkpoint import load_hypervisor, save_hypervisor
    from hypervisor import Hypervisor

    n = args.sessions
    caps = {"S": n + 1024, "D": 3 * n + 4096, "G": n + 1024, "T": n + 1024, "P": 4, "B": 1024 * n + (1 << 20)}
    st = GovernanceStore(args.device, caps=caps)
    hv = Hypervisor(store=st)
    t0 = time.perf_counter()
    run = asyncio.run(hv.run_pipelines(PipelineSpec(), n))
    t_run = time.perf_counter() - t0
    assert run.ok == n, run.ok
    d = args.dir or tempfile.mkdtemp(prefix="ahv-ck-")
    posted0 = st._c.info()["posted"]
    t0 = time.perf_counter()
    save_hypervisor(hv, os.path.join(d, "ck"))
    t_save = time.perf_counter() - t0
    save_cmds = st._c.info()["posted"] - posted0
    size = sum(os.path.getsize(os.path.join(d, "ck", f)) for f in os.listdir(os.path.join(d, "ck")))
    st2 = GovernanceStore(args.device, caps=caps)
    hv2 = Hypervisor(store=st2)
    posted1 = st2._c.info()["posted"]
    t0 = time.perf_counter()
    load_hypervisor(os.path.join(d, "ck"), hv=hv2)
    t_load = time.perf_counter() - t0
    load_cmds = st2._c.info()["posted"] - posted1
    # restored sessions are ordinary sessions: views, roots, audit in place
    sid = run.session_ids[n // 2]
    m = hv2.get_session(sid)
    ok = m.delta_engine.compute_merkle_root() == run.roots[sid] and m.delta_engine.verify_chain()
    rep = hv2.verify_audit(run.session_ids[:1000])
    if not args.dir:
        shutil.rmtree(d, ignore_errors=True)
    print(json.dumps({
        "bench": "columnar_checkpoint", "device": args.device, "sessions": n, "run_pipelines_s": round(t_run, 3),
        "save_s": round(t_save, 3), "save_store_commands": save_cmds, "load_s": round(t_load, 3),
        "load_store_commands": load_cmds, "bytes": size, "restored_view_ok": bool(ok),
        "audit_ok_1000": bool(rep.ok), "verify": "K10 chains + K09 roots over every restored session",
    }))


if __name__ == "__main__":
    main()
