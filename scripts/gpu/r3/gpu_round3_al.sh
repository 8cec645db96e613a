#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp AHV_SKIP_AUTOBUILD=1
OUT=gpurun_out/r3al
mkdir -p $OUT
timeout -k 10 200 python -u scripts/batch_api_prof.py > $OUT/prof.log 2>&1 || exit 1
echo done
