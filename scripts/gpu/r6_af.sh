#!/bin/bash
# Round 6, call af: Merkle roots folded into the chain lanes (chain_roots) on top of the
# render-first layout — batched pipeline GPU tests, hetero A/B, kernel stats.
#
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp AHV_SKIP_AUTOBUILD=1
OUT=gpurun_out/r6af
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_store_pipeline.py tests/test_batched_views.py tests/test_gpu_pipeline.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/tests.txt 2>&1; rc=$?
tail -2 $OUT/tests.txt; [ $rc -eq 0 ] || exit $rc
for cfg in "1 1" "1 0" "0 0"; do
  set -- $cfg
  for S in 1048576 4194304; do
    AHV_SP_OVERLAP=$1 AHV_SP_CHAIN_ROOTS=$2 timeout -k 10 300 python bench.py --mix hetero --no-scalar --no-api --sessions $S \
      --steps 10 --warmup 2 > $OUT/hetero_o$1r$2_$S.json 2>$OUT/hetero_o$1r$2_$S.err || exit $?
    echo "overlap=$1 chain_roots=$2 S=$S $(tail -1 $OUT/hetero_o$1r$2_$S.json | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python bench.py --mix hetero --no-scalar \
  --no-api --sessions 1048576 --steps 5 --warmup 1 > $OUT/prof.log 2>&1 || exit $?
f=$(find $OUT/prof -name "*kernel_stats.csv" | head -1); cp "$f" $OUT/kernel_stats.csv
cut -d, -f1-4 $OUT/kernel_stats.csv | head -8 | cut -c1-150
