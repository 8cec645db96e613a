#!/bin/bash
# Round 5, call ah: the close runs its root-independent work (row checks, leaf gather,
# state / participant / bond / retention writes) before waiting for the provisional
# tree — worker tests, root stress, awaited split and timeline.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp AHV_SKIP_AUTOBUILD=1
OUT=gpurun_out/r5ah
mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests/test_reference_trace.py tests/test_speculation.py tests/test_gpu_store.py \
  tests/test_api_concurrency.py tests/test_audit_verify.py -m gpu -x -q -p no:cacheprovider --timeout 300 \
  --timeout-method thread > $OUT/tests.log 2>&1; rc=$?
tail -2 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python scripts/root_stress.py 6000 cuda > $OUT/stress.txt 2>&1 || exit $?
tail -1 $OUT/stress.txt | cut -c1-200
timeout -k 10 300 python scripts/percall_split.py cuda > $OUT/split_awaited.txt 2>&1 || exit $?
grep -v amdgpu $OUT/split_awaited.txt | tail -12
AHV_SPEC_TERMINATE=0 timeout -k 10 300 python scripts/percall_timeline.py > $OUT/timeline_awaited.jsonl 2>&1 || exit $?
grep -v amdgpu $OUT/timeline_awaited.jsonl | grep -E "p50|SESS_CLOSE|tree" | cut -c1-300
