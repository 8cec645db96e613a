#!/bin/bash
# Round 5, call v: host CPU of the concurrent per-call path after the lazy
# engines / lazy VFS / native id words / batched close; API tests.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp AHV_SKIP_AUTOBUILD=1
OUT=gpurun_out/r5v
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_reference_trace.py tests/test_speculation.py tests/test_gpu_store.py \
  tests/test_api_concurrency.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1; rc=$?
tail -2 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
N=10000 TOP=45 timeout -k 10 300 python scripts/profile_gather.py > $OUT/gather_tot.txt 2>&1 || exit $?
N=10000 TOP=60 SORT=cumulative timeout -k 10 300 python scripts/profile_gather.py > $OUT/gather_cum.txt 2>&1 || exit $?
grep -v amdgpu $OUT/gather_tot.txt | head -3
timeout -k 10 300 python scripts/percall_split.py cuda > $OUT/split_awaited.txt 2>&1 || exit $?
grep -v amdgpu $OUT/split_awaited.txt | tail -12
