#!/bin/bash
# Round 4, call j: host-predicted terminate roots + per-session drain on the GPU:
# Store tests, the gather profile, worker probes, per-call, the bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp AHV_SKIP_AUTOBUILD=1
OUT=gpurun_out/r4j
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_store.py tests/test_gpu_store.py tests/test_store_fuzz.py tests/test_api_concurrency.py tests/test_speculation.py tests/test_reference_trace.py tests/test_checkpoint.py -m gpu -x -q -p no:cacheprovider \
  --timeout 120 --timeout-method thread > $OUT/pytest_store.log 2>&1 && echo store-tests-ok && \
N=10000 timeout -k 10 300 python scripts/profile_gather.py > $OUT/gather_dev.log 2>&1 && echo gather-ok && \
timeout -k 10 300 python scripts/probe_worker.py > $OUT/probe.log 2>&1 && echo probe-ok && \
ITERS=2000 timeout -k 10 300 python scripts/profile_percall.py > $OUT/percall.log 2>&1 && echo percall-ok && \
timeout -k 10 600 python bench.py --steps 10 --warmup 2 > $OUT/bench.log 2>&1 && echo bench-ok
rc=$?
tail -2 $OUT/pytest_store.log; head -2 $OUT/gather_dev.log; tail -1 $OUT/probe.log; grep p50_us $OUT/percall.log | cut -c1-200
tail -1 $OUT/bench.log | cut -c1-600
exit $rc
