#!/bin/bash
# Round 6, call ae: render-first batch layout (rows blocks interleaved with the prefix
# SHA blocks in one launch) — batched pipeline GPU tests, hetero bench A/B
# (AHV_SP_OVERLAP), kernel stats of the new layout.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp AHV_SKIP_AUTOBUILD=1
OUT=gpurun_out/r6ae
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_store_pipeline.py tests/test_batched_views.py tests/test_gpu_pipeline.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/tests.txt 2>&1; rc=$?
tail -2 $OUT/tests.txt; [ $rc -eq 0 ] || exit $rc
for ov in 1 0; do
  for S in 1048576 4194304; do
    AHV_SP_OVERLAP=$ov timeout -k 10 300 python bench.py --mix hetero --no-scalar --no-api --sessions $S --steps 10 --warmup 2 \
      > $OUT/hetero_o${ov}_$S.json 2>$OUT/hetero_o${ov}_$S.err || exit $?
    echo "overlap=$ov S=$S $(tail -1 $OUT/hetero_o${ov}_$S.json | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python bench.py --mix hetero --no-scalar \
  --no-api --sessions 1048576 --steps 5 --warmup 1 > $OUT/prof.log 2>&1 || exit $?
f=$(find $OUT/prof -name "*kernel_stats.csv" | head -1); cp "$f" $OUT/kernel_stats.csv
cut -d, -f1-4 $OUT/kernel_stats.csv | head -8 | cut -c1-150
