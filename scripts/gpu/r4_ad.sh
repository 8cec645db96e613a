#!/bin/bash
# Round 4, call ad: FREE_ROWS drains narrowed to the rows being freed (worker bit 16).
# Store/API GPU tests, then per-call outliers (slow-call wrappers) narrowed vs full
# drains, then per-call percentiles.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp AHV_SKIP_AUTOBUILD=1
OUT=gpurun_out/r4ad
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_store.py tests/test_gpu_store.py tests/test_store_fuzz.py tests/test_api_concurrency.py \
  tests/test_speculation.py tests/test_reference_trace.py tests/test_checkpoint.py tests/test_store_lifecycle.py -m gpu -x -q \
  -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 && echo tests-ok && \
timeout -k 10 300 python scripts/percall_outliers.py cuda 5000 > $OUT/outliers_narrow.txt 2>&1 && echo outliers-narrow-ok && \
AHV_STORE_NARROW_FREE=0 timeout -k 10 300 python scripts/percall_outliers.py cuda 5000 > $OUT/outliers_full.txt 2>&1 && echo outliers-full-ok && \
ITERS=5000 timeout -k 10 300 python scripts/profile_percall.py > $OUT/percall.log 2>&1 && echo percall-ok
rc=$?
tail -1 $OUT/pytest.log
head -9 $OUT/outliers_narrow.txt
head -9 $OUT/outliers_full.txt
grep p50_us $OUT/percall.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print({k: d[k] for k in ('p50_us','mean_us','p90_us','p99_us','max_us','host_cpu_us_per_pipeline')})"
exit $rc
