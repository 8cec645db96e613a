#!/bin/bash
# Round 6, call aj: sampled wall-clock profile of the 10^4-concurrent gather on the
# final build (device store and host engines), for the remaining per-pipeline costs.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp AHV_SKIP_AUTOBUILD=1
OUT=gpurun_out/r6aj
mkdir -p $OUT
DEV=cuda N=10000 timeout -k 10 200 python scripts/sample_gather.py > $OUT/sample_cuda.txt 2>&1 || exit $?
DEV=host N=10000 timeout -k 10 200 python scripts/sample_gather.py > $OUT/sample_host.txt 2>&1 || exit $?
head -3 $OUT/sample_cuda.txt; head -3 $OUT/sample_host.txt
