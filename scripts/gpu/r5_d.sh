#!/bin/bash
# Round 5, call d: is the reference-trace capture mismatch of r5c reproducible?  The
# trace test alone three times (separate processes); then the per-call worker timeline
# (AHV_STORE_TRACE) with device-awaited and speculated terminate roots, and the
# per-stage split, with the drop-time close no longer waiting.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp AHV_SKIP_AUTOBUILD=1
OUT=gpurun_out/r5d
mkdir -p $OUT
for k in 1 2 3; do
  timeout -k 10 300 python -u -m pytest tests/test_reference_trace.py -m gpu -x -q -p no:cacheprovider --timeout 240 \
    --timeout-method thread > $OUT/trace$k.log 2>&1; echo trace$k rc=$?
done
AHV_SPEC_TERMINATE=0 timeout -k 10 300 python scripts/percall_timeline.py > $OUT/timeline_awaited.jsonl 2>&1 && \
timeout -k 10 300 python scripts/percall_timeline.py > $OUT/timeline_spec.jsonl 2>&1 && \
AHV_SPEC_TERMINATE=0 timeout -k 10 300 python scripts/percall_split.py cuda > $OUT/split_awaited.txt 2>&1 && \
timeout -k 10 300 python scripts/percall_split.py cuda > $OUT/split_spec.txt 2>&1; echo profiles rc=$?
for k in 1 2 3; do tail -1 $OUT/trace$k.log; grep -E "^E  +#" $OUT/trace$k.log | head -3; done
grep -v amdgpu $OUT/timeline_awaited.jsonl; grep -v amdgpu $OUT/timeline_spec.jsonl | head -1
grep -v amdgpu $OUT/split_awaited.txt | tail -3; grep -v amdgpu $OUT/split_spec.txt | tail -3
