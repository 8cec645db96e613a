#!/bin/bash
# Round 4, call ac: which call inside create_session takes the ~7 ms outliers
# (store.alloc / post_expect / DeviceSession() / session_views timed when > 1 ms).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp AHV_SKIP_AUTOBUILD=1
OUT=gpurun_out/r4ac
mkdir -p $OUT
timeout -k 10 300 python scripts/percall_outliers.py cuda 5000 > $OUT/outliers.txt 2>&1 && echo outliers-ok
rc=$?
head -9 $OUT/outliers.txt
exit $rc
