#!/bin/bash
# Round 6, call i: cooperative small-batch template kernel (4 waves per 64 sessions) —
# oracle tests, config 2 step time, kernel stats.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp AHV_SKIP_AUTOBUILD=1
OUT=gpurun_out/r6i
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_headline_oracle.py -k cooperative -m gpu -x -q -p no:cacheprovider --timeout 240 --timeout-method thread > $OUT/tests_coop.log 2>&1; rc=$?
tail -3 $OUT/tests_coop.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python benchmarks/bench_configs.py config2 > $OUT/config2.jsonl 2> $OUT/config2.err || exit $?
cat $OUT/config2.jsonl
AHV_TEMPLATE_COOP=0 timeout -k 10 200 python benchmarks/bench_configs.py config2 > $OUT/config2_nocoop.jsonl 2>> $OUT/config2.err || exit $?
cat $OUT/config2_nocoop.jsonl
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o c2 -- python benchmarks/bench_configs.py config2 > $OUT/prof.log 2>&1 || exit $?
find $OUT/prof -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} $OUT/config2_kernel_stats.csv
head -8 $OUT/config2_kernel_stats.csv | cut -c1-200
