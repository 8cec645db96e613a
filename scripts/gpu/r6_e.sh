#!/bin/bash
# Round 6, call e: the worker's SHA-256 round / schedule loops out of line (one copy
# shared by its three waves; kernel code 240 → 193 KB): worker tests, root stress,
# per-call timeline and split.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp AHV_SKIP_AUTOBUILD=1 AHV_SPEC_TERMINATE=0
OUT=gpurun_out/r6e
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_reference_trace.py tests/test_speculation.py tests/test_gpu_store.py \
  tests/test_api_concurrency.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1; rc=$?
tail -2 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python scripts/root_stress.py 6000 cuda > $OUT/stress.txt 2>&1 || exit $?
tail -1 $OUT/stress.txt | cut -c1-200
timeout -k 10 200 python scripts/percall_timeline.py > $OUT/timeline.jsonl 2>&1 || exit $?
grep -E "p50|CAPTURE|CLOSE" $OUT/timeline.jsonl | cut -c1-330
timeout -k 10 200 python scripts/percall_split.py cuda > $OUT/split.txt 2>&1 || exit $?
grep -v amdgpu $OUT/split.txt | tail -11
