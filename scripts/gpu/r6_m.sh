#!/bin/bash
# Round 6, call m: coop kernel with the row writes moved off the chain; config 2
# through GovernanceEngine now with pre-rendered change fragments.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp AHV_SKIP_AUTOBUILD=1
OUT=gpurun_out/r6m
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_headline_oracle.py -k cooperative tests/test_graphs.py tests/test_gpu_pipeline.py -m gpu -x -q -p no:cacheprovider --timeout 240 --timeout-method thread > $OUT/tests.log 2>&1; rc=$?
tail -2 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python scripts/coop_phases.py 10000 > $OUT/coop_phases.json 2>&1 || exit $?
grep -E "hash r0|tail|root|events|render\"" $OUT/coop_phases.json
timeout -k 10 200 python benchmarks/bench_configs.py config2 > $OUT/config2.jsonl 2> $OUT/config2.err || exit $?
cat $OUT/config2.jsonl
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o c2 -- python benchmarks/bench_configs.py config2 > $OUT/prof.log 2>&1 || exit $?
f=$(find $OUT/prof -name "*kernel_stats.csv" | head -1); cp "$f" $OUT/config2_kernel_stats.csv
cut -d, -f1-4 $OUT/config2_kernel_stats.csv | head -5
