#!/bin/bash
# Round 6, call n: full GPU suite + the default 1-GPU bench after the coop kernel
# LDS hand-off (fresh container rebuild).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp AHV_SKIP_AUTOBUILD=1
OUT=gpurun_out/r6n
mkdir -p $OUT
timeout -k 10 800 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/gpu_tests.txt 2>&1; rc=$?
tail -3 $OUT/gpu_tests.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py > $OUT/bench.json 2> $OUT/bench.err || exit $?
tail -1 $OUT/bench.json | cut -c1-600
