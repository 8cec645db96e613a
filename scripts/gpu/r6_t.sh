#!/bin/bash
# Round 6, call t: deferred commitment engine + lazy ring enforcer; per-call
# timeline (worker trace) with the native control plane; gather; split.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp AHV_SKIP_AUTOBUILD=1
OUT=gpurun_out/r6t
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_speculation.py tests/test_gpu_store.py -m gpu -x -q -p no:cacheprovider --timeout 240 --timeout-method thread > $OUT/tests.txt 2>&1; rc=$?
tail -2 $OUT/tests.txt; [ $rc -eq 0 ] || exit $rc
N=10000 timeout -k 10 200 python scripts/profile_gather.py > $OUT/gather.txt 2>&1 || exit $?
DEV=cuda N=10000 timeout -k 10 200 python scripts/sample_gather.py > $OUT/sample_cuda.txt 2>&1 || exit $?
timeout -k 10 120 python scripts/percall_split.py cuda > $OUT/split.txt 2>&1 || exit $?
ITERS=400 timeout -k 10 200 python scripts/percall_timeline.py > $OUT/timeline.jsonl 2>&1 || exit $?
head -3 $OUT/gather.txt | grep pipelines_per_s | cut -c1-300; head -2 $OUT/sample_cuda.txt | tail -1; grep sum $OUT/split.txt
cat $OUT/timeline.jsonl | grep -v amdgpu | cut -c1-330
