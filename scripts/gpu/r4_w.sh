#!/bin/bash
# Round 4, call w: the per-call steady state is now bound by the hash-engine wave
# (≈60 µs per pipeline vs ≈58 µs of host work): A/B of the command wave computing
# every capture's prefix midstate (AHV_STORE_PREFIX_ALWAYS=1), which moves ≈half of
# each record's blocks off the engine.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp AHV_SKIP_AUTOBUILD=1
OUT=gpurun_out/r4w
mkdir -p $OUT
ITERS=3000 timeout -k 10 300 python scripts/profile_percall.py > $OUT/percall_def.log 2>&1 && echo def-ok && \
AHV_STORE_PREFIX_ALWAYS=1 ITERS=3000 timeout -k 10 300 python scripts/profile_percall.py > $OUT/percall_pa.log 2>&1 && echo pa-ok && \
AHV_STORE_PREFIX_ALWAYS=1 N=10000 timeout -k 10 300 python scripts/profile_gather.py > $OUT/gather_pa.log 2>&1 && echo gpa-ok && \
AHV_STORE_PREFIX_ALWAYS=1 timeout -k 10 300 python scripts/probe_worker.py > $OUT/probe_pa.log 2>&1 && echo probe-ok && \
AHV_STORE_PREFIX_ALWAYS=1 timeout -k 10 300 python -u -m pytest tests/test_store.py tests/test_speculation.py tests/test_gpu_store.py -m gpu -x -q \
  -p no:cacheprovider --timeout 200 --timeout-method thread > $OUT/pytest_pa.log 2>&1 && echo tests-ok
rc=$?
for f in percall_def percall_pa; do grep p50_us $OUT/$f.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$f', {k: d[k] for k in ('p50_us','mean_us','host_cpu_us_per_pipeline')}, d['store_info_delta'].get('engine_busy_us',0)/d['iters'], d['store_info_delta'].get('worker_busy_us',0)/d['iters'])"; done
head -3 $OUT/gather_pa.log | cut -c1-230; tail -1 $OUT/probe_pa.log; tail -1 $OUT/pytest_pa.log
exit $rc
