#!/bin/bash
# Round 6, call ah: lane renderer with the straight-line arena sink (AHV_SP_SINK) and
# register budgets for more waves per SIMD (AHV_SP_RENDER_WAVES / AHV_SP_CHAIN_WAVES):
# batch GPU tests, interleaved hetero A/B at 1 M sessions per step, kernel stats.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp AHV_SKIP_AUTOBUILD=1
OUT=gpurun_out/r6ah
mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests/test_store_pipeline.py tests/test_gpu_pipeline.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/tests.txt 2>&1; rc=$?
tail -2 $OUT/tests.txt; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for cfg in "staged 1 1" "flat 1 1" "flat 5 1" "flat 6 1" "flat 1 4" "flat 1 5"; do
    set -- $cfg
    AHV_SP_SINK=$1 AHV_SP_RENDER_WAVES=$2 AHV_SP_CHAIN_WAVES=$3 timeout -k 10 300 python bench.py --mix hetero --no-scalar --no-api \
      --sessions 1048576 --steps 20 --warmup 3 > $OUT/h_$1_$2_$3_$rep.json 2>$OUT/h_$1_$2_$3_$rep.err || exit $?
    echo "rep=$rep sink=$1 render_waves=$2 chain_waves=$3 $(tail -1 $OUT/h_$1_$2_$3_$rep.json | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
for cfg in "staged 1 1" "flat 1 1"; do
  set -- $cfg
  AHV_SP_SINK=$1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_$1 -o run --output-format csv -- python bench.py --mix hetero \
    --no-scalar --no-api --sessions 1048576 --steps 5 --warmup 1 > $OUT/prof_$1.log 2>&1 || exit $?
  f=$(find $OUT/prof_$1 -name "*kernel_stats.csv" | head -1); cp "$f" $OUT/kernel_stats_$1.csv
done
