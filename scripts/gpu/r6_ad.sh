#!/bin/bash
# Round 6, call ad: full GPU suite + default bench + headline kernel stats on the final build
# (validates the store transport slot-trim / kept-array changes on the GPU).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp AHV_SKIP_AUTOBUILD=1
OUT=gpurun_out/r6ad
mkdir -p $OUT
timeout -k 10 800 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/gpu_tests.txt 2>&1; rc=$?
tail -3 $OUT/gpu_tests.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py > $OUT/bench.json 2> $OUT/bench.err || exit $?
tail -1 $OUT/bench.json | cut -c1-400
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o hl -- python bench.py --steps 5 --warmup 2 --no-scalar --no-api > $OUT/prof.log 2>&1 || exit $?
f=$(find $OUT/prof -name "*kernel_stats.csv" | head -1); cp "$f" $OUT/headline_kernel_stats.csv
cut -d, -f1-4 $OUT/headline_kernel_stats.csv | head -6 | cut -c1-160
