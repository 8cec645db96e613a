#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp AHV_SKIP_AUTOBUILD=1
OUT=gpurun_out/r3ag
mkdir -p $OUT
timeout -k 10 120 python -u scripts/engine_probe.py 500 > $OUT/engine.json 2> $OUT/err.log || exit 1
echo done
