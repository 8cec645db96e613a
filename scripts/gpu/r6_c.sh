#!/bin/bash
# Round 6, call c: per-call timeline A/B — prefix wave on/off (is c0's hash slowed
# by the prefix wave running beside it?).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp AHV_SKIP_AUTOBUILD=1 AHV_SPEC_TERMINATE=0
OUT=gpurun_out/r6c
mkdir -p $OUT
AHV_STORE_PREFIX=0 timeout -k 10 200 python scripts/percall_timeline.py > $OUT/timeline_noprefix.jsonl 2>&1 || exit $?
grep -E "p50|CAPTURE|CLOSE" $OUT/timeline_noprefix.jsonl | cut -c1-330
timeout -k 10 200 python scripts/percall_timeline.py > $OUT/timeline_prefix.jsonl 2>&1 || exit $?
grep -E "p50|CAPTURE|CLOSE" $OUT/timeline_prefix.jsonl | cut -c1-330
