#!/bin/bash
# Round 4, call af: command-wave throughput — light result publication (bit 32: vmcnt
# wait instead of a system release with L2 write-back per command) and next-slot
# prefetch (bit 64).  Store/API GPU tests with both on; worker lag and per-call
# percentiles for off / light / prefetch / both; per-call + gather for both vs off.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp AHV_SKIP_AUTOBUILD=1
OUT=gpurun_out/r4af
mkdir -p $OUT
AHV_STORE_LIGHT_PUBLISH=1 AHV_STORE_SLOT_PREFETCH=1 timeout -k 10 600 python -u -m pytest tests/test_store.py tests/test_gpu_store.py \
  tests/test_store_fuzz.py tests/test_api_concurrency.py tests/test_speculation.py tests/test_reference_trace.py tests/test_checkpoint.py \
  tests/test_store_lifecycle.py tests/test_store_pipeline.py -m gpu -x -q \
  -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/pytest_both.log 2>&1 && echo tests-ok && \
timeout -k 10 300 python scripts/percall_outliers.py cuda 5000 > $OUT/ol_off.txt 2>&1 && echo o1 && \
AHV_STORE_LIGHT_PUBLISH=1 timeout -k 10 300 python scripts/percall_outliers.py cuda 5000 > $OUT/ol_light.txt 2>&1 && echo o2 && \
AHV_STORE_SLOT_PREFETCH=1 timeout -k 10 300 python scripts/percall_outliers.py cuda 5000 > $OUT/ol_prefetch.txt 2>&1 && echo o3 && \
AHV_STORE_LIGHT_PUBLISH=1 AHV_STORE_SLOT_PREFETCH=1 timeout -k 10 300 python scripts/percall_outliers.py cuda 5000 > $OUT/ol_both.txt 2>&1 && echo o4 && \
AHV_STORE_LIGHT_PUBLISH=1 AHV_STORE_SLOT_PREFETCH=1 ITERS=5000 timeout -k 10 300 python scripts/profile_percall.py > $OUT/percall_both.log 2>&1 && echo p1 && \
AHV_STORE_LIGHT_PUBLISH=1 AHV_STORE_SLOT_PREFETCH=1 N=10000 timeout -k 10 300 python scripts/profile_gather.py > $OUT/gather_both.log 2>&1 && echo g1 && \
N=10000 timeout -k 10 300 python scripts/profile_gather.py > $OUT/gather_off.log 2>&1 && echo g2
rc=$?
tail -1 $OUT/pytest_both.log
for f in ol_off ol_light ol_prefetch ol_both; do echo "== $f"; sed -n 2,5p $OUT/$f.txt | cut -c1-160; done
grep p50_us $OUT/percall_both.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print({k: d[k] for k in ('p50_us','mean_us','p90_us','p99_us','max_us','host_cpu_us_per_pipeline')})"
for f in gather_both gather_off; do sed -n 2,3p $OUT/$f.log | cut -c1-230; done
exit $rc
