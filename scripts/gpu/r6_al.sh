#!/bin/bash
# Round 6, call al: the hetero batch as two halves whose passes overlap on two streams
# (store_pipeline.launch_pair, bench.py --sp-split 2) vs one batch — interleaved A/B,
# batch GPU tests, kernel trace of the split step.
# (The split path was removed again after this A/B: no gain — kernels of the two halves
# overlapped in the trace but each ran correspondingly slower; profiles/r6/hetero_split_ab_r6al.txt.)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp AHV_SKIP_AUTOBUILD=1
OUT=gpurun_out/r6al
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_store_pipeline.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/tests.txt 2>&1; rc=$?
tail -2 $OUT/tests.txt; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for sp in 1 2; do
    for S in 1048576 4194304; do
      timeout -k 10 300 python bench.py --mix hetero --no-scalar --no-api --sessions $S --steps 20 --warmup 3 --sp-split $sp \
        > $OUT/h_s${sp}_${S}_$rep.json 2>$OUT/h_s${sp}_${S}_$rep.err || exit $?
      echo "rep=$rep split=$sp S=$S $(tail -1 $OUT/h_s${sp}_${S}_$rep.json | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
    done
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python bench.py --mix hetero --no-scalar \
  --no-api --sessions 1048576 --steps 5 --warmup 1 --sp-split 2 > $OUT/prof.log 2>&1 || exit $?
f=$(find $OUT/prof -name "*kernel_stats.csv" | head -1); cp "$f" $OUT/kernel_stats.csv
f=$(find $OUT/prof -name "*kernel_trace.csv" | head -1); cp "$f" $OUT/kernel_trace.csv
