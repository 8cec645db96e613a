#!/bin/bash
# Round 4, call af: light result publication on the command wave (worker bit 32:
# vmcnt wait instead of a system release with L2 write-back per command) — store/API
# GPU tests with it on, worker lag + per-call percentiles on vs off, gather on vs off.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp AHV_SKIP_AUTOBUILD=1
OUT=gpurun_out/r4af
mkdir -p $OUT
AHV_STORE_LIGHT_PUBLISH=1 timeout -k 10 600 python -u -m pytest tests/test_store.py tests/test_gpu_store.py tests/test_store_fuzz.py \
  tests/test_api_concurrency.py tests/test_speculation.py tests/test_reference_trace.py tests/test_checkpoint.py \
  tests/test_store_lifecycle.py tests/test_store_pipeline.py -m gpu -x -q \
  -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/pytest_light.log 2>&1 && echo tests-ok && \
AHV_STORE_LIGHT_PUBLISH=1 timeout -k 10 300 python scripts/percall_outliers.py cuda 5000 > $OUT/outliers_light.txt 2>&1 && echo ol-ok && \
timeout -k 10 300 python scripts/percall_outliers.py cuda 5000 > $OUT/outliers_full.txt 2>&1 && echo of-ok && \
AHV_STORE_LIGHT_PUBLISH=1 ITERS=5000 timeout -k 10 300 python scripts/profile_percall.py > $OUT/percall_light.log 2>&1 && echo pl-ok && \
AHV_STORE_LIGHT_PUBLISH=1 N=10000 timeout -k 10 300 python scripts/profile_gather.py > $OUT/gather_light.log 2>&1 && echo gl-ok && \
N=10000 timeout -k 10 300 python scripts/profile_gather.py > $OUT/gather_full.log 2>&1 && echo gf-ok
rc=$?
tail -1 $OUT/pytest_light.log
for f in outliers_light outliers_full; do echo "== $f"; sed -n 2,7p $OUT/$f.txt | cut -c1-200; done
grep p50_us $OUT/percall_light.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print({k: d[k] for k in ('p50_us','mean_us','p90_us','p99_us','max_us','host_cpu_us_per_pipeline')})"
for f in gather_light gather_full; do sed -n 2,3p $OUT/$f.log | cut -c1-260; done
exit $rc
