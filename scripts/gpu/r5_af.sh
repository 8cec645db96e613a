#!/bin/bash
# Round 5, call af: where config 2's 0.13 ms step goes (kernel trace).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp AHV_SKIP_AUTOBUILD=1
OUT=gpurun_out/r5af
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python benchmarks/bench_configs.py config2 \
  > $OUT/prof.log 2>&1 || exit $?
grep -v amdgpu $OUT/prof.log | grep config2 | cut -c1-300
head -12 $OUT/prof/run_kernel_stats.csv | cut -c1-200
