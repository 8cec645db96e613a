#!/bin/bash
# Round 5, call t: terminate overlaps its host bookkeeping with the device close —
# worker/API tests, the per-call split and p50, then BASELINE configs 2-5.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp AHV_SKIP_AUTOBUILD=1
OUT=gpurun_out/r5t
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_reference_trace.py tests/test_speculation.py tests/test_gpu_store.py \
  tests/test_api_concurrency.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1; rc=$?
tail -2 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/percall_split.py cuda > $OUT/split_awaited.txt 2>&1 || exit $?
grep -v amdgpu $OUT/split_awaited.txt | tail -12
timeout -k 10 400 python benchmarks/bench_configs.py config2 config3 config4 config5 > $OUT/configs.jsonl 2>&1 || exit $?
grep -v amdgpu $OUT/configs.jsonl | tail -6 | cut -c1-300
