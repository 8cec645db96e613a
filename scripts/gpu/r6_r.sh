#!/bin/bash
# Round 6, call r: native finalisers + command ring size A/B (AHV_STORE_SLOTS) on
# the 10^4-concurrent gather; sampled profile; per-call split and p50.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp AHV_SKIP_AUTOBUILD=1
OUT=gpurun_out/r6r
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_speculation.py tests/test_gpu_store.py -m gpu -x -q -p no:cacheprovider --timeout 240 --timeout-method thread > $OUT/tests.txt 2>&1; rc=$?
tail -2 $OUT/tests.txt; [ $rc -eq 0 ] || exit $rc
for slots in 4096 32768; do
  AHV_STORE_SLOTS=$slots N=10000 timeout -k 10 200 python scripts/profile_gather.py > $OUT/gather_s$slots.txt 2>&1 || exit $?
done
AHV_STORE_SLOTS=32768 DEV=cuda N=10000 timeout -k 10 200 python scripts/sample_gather.py > $OUT/sample_cuda.txt 2>&1 || exit $?
timeout -k 10 120 python scripts/percall_split.py cuda > $OUT/split.txt 2>&1 || exit $?
ITERS=2000 timeout -k 10 200 python scripts/profile_percall.py > $OUT/percall.txt 2>&1 || exit $?
for f in $OUT/gather_s*.txt; do echo $f; head -3 $f | grep pipelines_per_s | cut -c1-330; done
head -2 $OUT/sample_cuda.txt; grep sum $OUT/split.txt; head -2 $OUT/percall.txt | tail -1 | cut -c1-200
