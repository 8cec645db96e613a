#!/bin/bash
# Round 6, call ac: kept results in a per-slot array (no hash-map node per posted
# command), expectation checks in place — store GPU tests, root stress, gather, p50.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp AHV_SKIP_AUTOBUILD=1
OUT=gpurun_out/r6ac
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_speculation.py tests/test_gpu_store.py tests/test_store.py -m gpu -x -q -p no:cacheprovider --timeout 240 --timeout-method thread > $OUT/tests.txt 2>&1; rc=$?
tail -2 $OUT/tests.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python scripts/root_stress.py 6000 cuda > $OUT/root_stress.txt 2>&1 || exit $?
tail -1 $OUT/root_stress.txt | cut -c1-120
for r in 1 2; do
  N=10000 timeout -k 10 200 python scripts/profile_gather.py > $OUT/gather$r.txt 2>&1 || exit $?
  head -3 $OUT/gather$r.txt | grep pipelines_per_s | cut -c1-200
done
ITERS=2000 timeout -k 10 200 python scripts/profile_percall.py > $OUT/percall.txt 2>&1 || exit $?
head -2 $OUT/percall.txt | tail -1 | cut -c1-160
