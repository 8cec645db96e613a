#!/bin/bash
# Round 6, call ab: sampled profile of the 10^4-concurrent gather on the current build.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp AHV_SKIP_AUTOBUILD=1
OUT=gpurun_out/r6ab
mkdir -p $OUT
DEV=cuda N=10000 timeout -k 10 200 python scripts/sample_gather.py > $OUT/sample_cuda.txt 2>&1 || exit $?
N=10000 timeout -k 10 200 python scripts/profile_gather.py > $OUT/gather.txt 2>&1 || exit $?
head -2 $OUT/sample_cuda.txt | tail -1; head -3 $OUT/gather.txt | grep pipelines_per_s | cut -c1-200
