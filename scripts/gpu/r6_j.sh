#!/bin/bash
# Round 6, call j: config 2 kernel stats (cooperative small-batch kernel).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp AHV_SKIP_AUTOBUILD=1
OUT=gpurun_out/r6j
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o c2 -- python benchmarks/bench_configs.py config2 > $OUT/prof.log 2>&1 || exit $?
f=$(find $OUT/prof -name "*kernel_stats.csv" | head -1); cp "$f" $OUT/config2_kernel_stats.csv
cut -d, -f1-8 $OUT/config2_kernel_stats.csv | head -10
