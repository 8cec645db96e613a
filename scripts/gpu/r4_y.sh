#!/bin/bash
# Round 4, call y: the per-call tail (mean 79 µs vs p50 58 µs) — latency percentiles,
# collector time and the slowest pipelines' slow calls.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp AHV_SKIP_AUTOBUILD=1
OUT=gpurun_out/r4y
mkdir -p $OUT
ITERS=3000 timeout -k 10 300 python scripts/profile_percall.py > $OUT/percall.log 2>&1 && echo percall-ok && \
timeout -k 10 300 python scripts/percall_outliers.py cuda 3000 > $OUT/outliers.txt 2>&1 && echo outliers-ok && \
ITERS=1000 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt -o kt -- python3 scripts/profile_percall.py > $OUT/kt.log 2>&1 && echo kt-ok && \
python scripts/prof_summary.py $(find $OUT/kt -name "*.db" | head -1) > $OUT/percall_kernel_trace.md
rc=$?
rm -rf $OUT/kt
grep p50_us $OUT/percall.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print({k: d[k] for k in ('p50_us','mean_us','p90_us','p99_us','max_us','gc_collections','gc_us_per_pipeline')})"
cat $OUT/outliers.txt
head -8 $OUT/percall_kernel_trace.md | cut -c1-200
exit $rc
