#!/bin/bash
# Round 6, call h: per-call timeline with the helper waves' jobs traced.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp AHV_SKIP_AUTOBUILD=1 AHV_SPEC_TERMINATE=0
OUT=gpurun_out/r6h
mkdir -p $OUT
timeout -k 10 200 python scripts/percall_timeline.py > $OUT/timeline.jsonl 2>&1 || exit $?
grep -E "p50|CAPTURE|CLOSE" $OUT/timeline.jsonl | cut -c1-420
