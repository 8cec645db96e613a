#!/bin/bash
# Round 6, call q: expectation cap non-blocking; sampled profiles (wall-clock
# timer) of the 10^4-concurrent gather, device store vs host engines.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp AHV_SKIP_AUTOBUILD=1
OUT=gpurun_out/r6q
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_speculation.py tests/test_gpu_store.py -m gpu -x -q -p no:cacheprovider --timeout 240 --timeout-method thread > $OUT/tests.txt 2>&1; rc=$?
tail -2 $OUT/tests.txt; [ $rc -eq 0 ] || exit $rc
N=10000 timeout -k 10 200 python scripts/profile_gather.py > $OUT/gather.txt 2>&1 || exit $?
DEV=cuda N=10000 timeout -k 10 200 python scripts/sample_gather.py > $OUT/sample_cuda.txt 2>&1 || exit $?
DEV=host N=10000 timeout -k 10 200 python scripts/sample_gather.py > $OUT/sample_host.txt 2>&1 || exit $?
timeout -k 10 120 python scripts/percall_split.py cuda > $OUT/split.txt 2>&1 || exit $?
head -2 $OUT/gather.txt | cut -c1-250; head -1 $OUT/sample_cuda.txt; head -1 $OUT/sample_host.txt; grep sum $OUT/split.txt
