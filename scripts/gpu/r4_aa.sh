#!/bin/bash
# Round 4, call aa: delta reclaim in batches of 4,096 — store/API GPU tests incl. the
# reference trace, per-call percentiles and outliers, the default bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp AHV_SKIP_AUTOBUILD=1
OUT=gpurun_out/r4aa
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_store.py tests/test_gpu_store.py tests/test_store_fuzz.py tests/test_api_concurrency.py \
  tests/test_speculation.py tests/test_reference_trace.py tests/test_checkpoint.py tests/test_store_lifecycle.py -m gpu -x -q \
  -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 && echo tests-ok && \
ITERS=5000 timeout -k 10 300 python scripts/profile_percall.py > $OUT/percall.log 2>&1 && echo percall-ok && \
timeout -k 10 300 python scripts/percall_outliers.py cuda 5000 > $OUT/outliers.txt 2>&1 && echo outliers-ok && \
timeout -k 10 600 python bench.py > $OUT/bench.log 2>&1 && echo bench-ok
rc=$?
tail -1 $OUT/pytest.log
grep p50_us $OUT/percall.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print({k: d[k] for k in ('p50_us','mean_us','p90_us','p99_us','max_us','host_cpu_us_per_pipeline')})"
head -4 $OUT/outliers.txt
tail -1 $OUT/bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print({k: d.get(k) for k in ('value','device_p50_us','device_mean_us','scalar_p50_us','api_gather_pipelines_per_s')})"
exit $rc
