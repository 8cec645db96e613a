#!/bin/bash
# Per-call gather throughput after the bounded poll pass; cProfile of the device gather.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp AHV_SKIP_AUTOBUILD=1
OUT=gpurun_out/r3u2
mkdir -p $OUT
timeout -k 10 400 python -u scripts/gather_prof.py cuda > $OUT/gather.log 2>&1 || exit 1
echo done
