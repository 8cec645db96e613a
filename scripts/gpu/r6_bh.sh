#!/bin/bash
# Round 6, call bh: config 5 with the re-chain prefix lanes keeping the next block's loads in
# flight (chain_prefix_kernel 89 -> 106 VGPRs): 338.6 vs 337.9 us, no gain — reverted.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp AHV_SKIP_AUTOBUILD=1
OUT=gpurun_out/r6bh
mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests/test_config5_arena.py tests/test_gpu_kernels.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/tests.txt 2>&1; rc=$?
tail -2 $OUT/tests.txt; [ $rc -eq 0 ] || exit $rc
for rep in 1 2 3; do
  timeout -k 10 300 python benchmarks/bench_configs.py config5 > $OUT/c5_$rep.jsonl 2> $OUT/c5_$rep.err || exit $?
  echo "rep=$rep $(python -c 'import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d["ms_per_storm"])' $OUT/c5_$rep.jsonl)"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python benchmarks/bench_configs.py config5 \
  > $OUT/prof.log 2>&1 || exit $?
f=$(find $OUT/prof -name "*kernel_stats.csv" | head -1); cp "$f" $OUT/kernel_stats.csv
