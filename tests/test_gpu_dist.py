"""The multi-rank bench path on a real GPU: ``bench.py`` under
``torch.distributed.run`` with ``AHV_BENCH_FORCE_DIST=1`` takes the exact code the
driver's 8-GPU scaling run executes — RCCL process group bound to the device,
double-buffered async X04 all-reduce, barriers, max-over-ranks timing — with
one rank, eager and hipGraph-replay forms (the graph captures the collective
through the C++ RCCL communicator)."""

from __future__ import annotations

import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


# --standalone: the rendezvous binds a port the OS picks at bind time (a port probed
# here and bound later by torchrun can be taken in between: EADDRINUSE)
_LAUNCH = ["-m", "torch.distributed.run", "--standalone", "--local-addr", "127.0.0.1", "--nnodes=1",
           "--nproc-per-node", "1"]


@pytest.mark.parametrize("graph", [False, True])
def test_bench_rccl_path_one_rank(cuda_device, graph):
    env = dict(os.environ, AHV_BENCH_FORCE_DIST="1", AHV_SKIP_AUTOBUILD="1")
    cmd = [sys.executable, *_LAUNCH, os.path.join(ROOT, "bench.py"),
           "--gpus", "1", "--sessions", "65536", "--agents", "65536", "--steps", "3", "--warmup", "1",
           "--no-scalar"] + (["--graph"] if graph else [])
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=240, env=env, cwd=ROOT)
    assert p.returncode == 0, p.stderr[-3000:]
    out = json.loads([l for l in p.stdout.splitlines() if l.startswith("{")][-1])
    assert out["n_gpus"] == 1 and out["last_step_counters"]["sessions"] == 65536
    assert out["last_step_counters"]["ok"] == 65536 and out["value"] > 0


def test_sharded_hypervisor_rccl_one_rank(cuda_device):
    """The sharded front-end's collectives (X01/X04/X05 on RCCL, control on gloo)
    with the device store, under torch.distributed.run — the 8-GPU code path."""
    env = dict(os.environ, AHV_SKIP_AUTOBUILD="1", PYTHONPATH=ROOT)
    cmd = [sys.executable, *_LAUNCH, os.path.join(ROOT, "scripts", "sharded_rccl_check.py")]
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=240, env=env, cwd=ROOT)
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-3000:]
    out = json.loads([l for l in p.stdout.splitlines() if l.startswith("{")][-1])
    assert out["ok"] and out["backend"] == "nccl" and out["store_gpu"]


def test_bench_hetero_mix_gfx950(cuda_device):
    """``bench.py --mix hetero`` on the GPU: the public batched API's kernels over
    store rows, re-run every step; outcomes identical across re-runs."""
    env = dict(os.environ, AHV_SKIP_AUTOBUILD="1")
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--mix", "hetero", "--sessions", "65536",
           "--agents", "65536", "--steps", "3", "--warmup", "1", "--no-scalar", "--no-api"]
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=240, env=env, cwd=ROOT)
    assert p.returncode == 0, p.stderr[-3000:]
    out = json.loads([l for l in p.stdout.splitlines() if l.startswith("{")][-1])
    assert out["mix"] == "hetero" and out["last_step_counters"]["sessions"] == 65536 and out["value"] > 0
