#!/bin/bash
# Round 5, call f: the store worker's prefix wave (wave 2) — worker oracle tests, then the
# per-call timeline (awaited and speculated terminate) with tree / wait instrumentation;
# headline step kernel trace (full vs emission-only A/B) for the kernel's share of the step.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp AHV_SKIP_AUTOBUILD=1
OUT=gpurun_out/r5f
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_reference_trace.py tests/test_speculation.py tests/test_gpu_store.py -m gpu -x -q \
  -p no:cacheprovider --timeout 240 --timeout-method thread > $OUT/worker_tests.log 2>&1; rc=$?
tail -3 $OUT/worker_tests.log; [ $rc -eq 0 ] || exit $rc
AHV_SPEC_TERMINATE=0 timeout -k 10 300 python scripts/percall_timeline.py > $OUT/timeline_awaited.jsonl 2>&1 && \
timeout -k 10 300 python scripts/percall_timeline.py > $OUT/timeline_spec.jsonl 2>&1 && \
AHV_SPEC_TERMINATE=0 timeout -k 10 300 python scripts/percall_split.py cuda > $OUT/split_awaited.txt 2>&1 && \
timeout -k 10 300 python scripts/percall_split.py cuda > $OUT/split_spec.txt 2>&1; rc=$?
grep -v amdgpu $OUT/timeline_awaited.jsonl; grep -v amdgpu $OUT/timeline_spec.jsonl | head -2
grep -v amdgpu $OUT/split_awaited.txt | tail -3; grep -v amdgpu $OUT/split_spec.txt | tail -3
[ $rc -eq 0 ] || exit $rc
for ab in 0 12; do
  AHV_TEMPLATE_AB=$ab timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_ab$ab -o run -- \
    python bench.py --steps 5 --warmup 1 --no-scalar --no-api --verify-sessions 0 > $OUT/prof_ab$ab.log 2>&1 || exit $?
  echo "ab=$ab done"
done
find $OUT -name "*kernel_stats.csv" | head
