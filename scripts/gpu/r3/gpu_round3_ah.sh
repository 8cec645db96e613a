#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp AHV_SKIP_AUTOBUILD=1
OUT=gpurun_out/r3ah
mkdir -p $OUT
timeout -k 10 200 python -u scripts/engine_clock_probe.py > $OUT/clock.json 2> $OUT/err.log || { tail -5 $OUT/err.log; exit 1; }
echo done
