#!/bin/bash
# Round 6, call b: BASELINE config 5 as stated (+ the 10 % subset line), config 2,
# and the per-call baseline (split, timeline, host-CPU profile) before the r6 work.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp AHV_SKIP_AUTOBUILD=1
OUT=gpurun_out/r6b
mkdir -p $OUT
timeout -k 10 300 python benchmarks/bench_configs.py config5 config5_subset config2 > $OUT/configs.jsonl 2> $OUT/configs.err || exit $?
cut -c1-400 $OUT/configs.jsonl
timeout -k 10 200 python scripts/percall_split.py cuda > $OUT/split_awaited.txt 2>&1 || exit $?
timeout -k 10 200 python scripts/percall_split.py host > $OUT/split_host.txt 2>&1 || exit $?
grep -v amdgpu $OUT/split_awaited.txt | tail -11
AHV_SPEC_TERMINATE=0 timeout -k 10 200 python scripts/percall_timeline.py > $OUT/timeline_awaited.jsonl 2>&1 || exit $?
DEV=cuda ITERS=3000 timeout -k 10 200 python scripts/profile_percall.py > $OUT/profile_percall.txt 2>&1 || exit $?
DEV=host ITERS=3000 timeout -k 10 200 python scripts/profile_percall.py > $OUT/profile_percall_host.txt 2>&1 || exit $?
echo done
