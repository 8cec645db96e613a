#!/bin/bash
# Round 6, call bf: the rows lanes' early loads reverted (they spilled the render+rows kernel: 68 B of
# scratch) — hoisted render loads (1) vs in line (0), kernel stats; compare render+rows with call bd.
#
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp AHV_SKIP_AUTOBUILD=1
OUT=gpurun_out/r6bf
mkdir -p $OUT
for rep in 1 2 3; do
  for h in 1 0; do
    AHV_SP_HOIST=$h timeout -k 10 300 python bench.py --mix hetero --no-scalar --no-api --sessions 1048576 --steps 20 --warmup 3 \
      > $OUT/h_h${h}_$rep.json 2>$OUT/h_h${h}_$rep.err || exit $?
    echo "rep=$rep hoist=$h $(tail -1 $OUT/h_h${h}_$rep.json | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
for h in 1 0; do
  AHV_SP_HOIST=$h timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof$h -o run --output-format csv -- python bench.py --mix hetero \
    --no-scalar --no-api --sessions 1048576 --steps 5 --warmup 1 > $OUT/prof$h.log 2>&1 || exit $?
  f=$(find $OUT/prof$h -name "*kernel_stats.csv" | head -1); cp "$f" $OUT/kernel_stats_h$h.csv
done
