#!/bin/bash
# Round 4, call ab: what makes the ~7 ms create_session outliers of the per-call
# device path (gen-2 collections? worker relaunches?) — outliers with GC and
# worker-launch telemetry, default collector thresholds and tune_gc().
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp AHV_SKIP_AUTOBUILD=1
OUT=gpurun_out/r4ab
mkdir -p $OUT
timeout -k 10 300 python scripts/percall_outliers.py cuda 5000 > $OUT/outliers.txt 2>&1 && echo outliers-ok && \
TUNE_GC=1 timeout -k 10 300 python scripts/percall_outliers.py cuda 5000 > $OUT/outliers_tunegc.txt 2>&1 && echo outliers-tune-ok
rc=$?
head -8 $OUT/outliers.txt
head -8 $OUT/outliers_tunegc.txt
exit $rc
