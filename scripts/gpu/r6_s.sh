#!/bin/bash
# Round 6, call s: batched heterogeneous pipelines with record heads rendered once
# per distinct (agent, changes) (C.frag_pack) — GPU batch tests, hetero bench
# A/B (AHV_SP_FRAGS), kernel stats.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp AHV_SKIP_AUTOBUILD=1
OUT=gpurun_out/r6s
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_store_pipeline.py tests/test_batched_views.py tests/test_gpu_pipeline.py -m gpu -x -q -p no:cacheprovider --timeout 240 --timeout-method thread > $OUT/tests.txt 2>&1; rc=$?
tail -2 $OUT/tests.txt; [ $rc -eq 0 ] || exit $rc
for fr in 1 0; do
  for S in 1048576 4194304; do
    AHV_SP_FRAGS=$fr timeout -k 10 300 python bench.py --mix hetero --no-scalar --no-api --sessions $S --steps 10 --warmup 2 \
      > $OUT/hetero_f${fr}_$S.json 2>$OUT/hetero_f${fr}_$S.err || exit $?
    echo "frags=$fr S=$S $(tail -1 $OUT/hetero_f${fr}_$S.json | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python bench.py --mix hetero --no-scalar \
  --no-api --sessions 1048576 --steps 5 --warmup 1 > $OUT/prof.log 2>&1 || exit $?
f=$(find $OUT/prof -name "*kernel_stats.csv" | head -1); cp "$f" $OUT/kernel_stats.csv
cut -d, -f1-4 $OUT/kernel_stats.csv | head -8 | cut -c1-150
