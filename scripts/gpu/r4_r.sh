#!/bin/bash
# Round 4, call r: host cost of the store's native entry points one call at a time.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp AHV_SKIP_AUTOBUILD=1
OUT=gpurun_out/r4r
mkdir -p $OUT
timeout -k 10 300 python scripts/probe_calls.py > $OUT/probe_calls.log 2>&1 && echo probe-ok && \
AHV_STORE_RING=host timeout -k 10 300 python scripts/probe_calls.py > $OUT/probe_calls_hostring.log 2>&1 && echo probe-h-ok
rc=$?
tail -1 $OUT/probe_calls.log; tail -1 $OUT/probe_calls_hostring.log
exit $rc
