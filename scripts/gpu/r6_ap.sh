#!/bin/bash
# Round 6, call ap: kernel stats of BASELINE config 5 (slash storm over every session +
# sigma_eff + full re-chain / Merkle of 625 k sessions) — where its 2.45 ms go.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp AHV_SKIP_AUTOBUILD=1
OUT=gpurun_out/r6ap
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python benchmarks/bench_configs.py config5 \
  > $OUT/prof.log 2>&1 || exit $?
f=$(find $OUT/prof -name "*kernel_stats.csv" | head -1); cp "$f" $OUT/kernel_stats.csv
grep config5 $OUT/prof.log | cut -c1-200
