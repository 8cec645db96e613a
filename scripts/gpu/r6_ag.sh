#!/bin/bash
# Round 6, call ag: interleaved hetero A/B of the render-first layout (AHV_SP_OVERLAP)
# and chain-lane Merkle roots (AHV_SP_CHAIN_ROOTS), two rounds of each on one box,
# plus kernel stats of the K09-kernel variant for a same-box comparison.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp AHV_SKIP_AUTOBUILD=1
OUT=gpurun_out/r6ag
mkdir -p $OUT
for rep in 1 2; do
  for cfg in "1 1" "1 0" "0 0" "0 1"; do
    set -- $cfg
    for S in 1048576 4194304; do
      AHV_SP_OVERLAP=$1 AHV_SP_CHAIN_ROOTS=$2 timeout -k 10 300 python bench.py --mix hetero --no-scalar --no-api --sessions $S \
        --steps 20 --warmup 3 > $OUT/h_o$1r$2_${S}_$rep.json 2>$OUT/h_o$1r$2_${S}_$rep.err || exit $?
      echo "rep=$rep overlap=$1 chain_roots=$2 S=$S $(tail -1 $OUT/h_o$1r$2_${S}_$rep.json | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
    done
  done
done
AHV_SP_CHAIN_ROOTS=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python bench.py --mix hetero --no-scalar \
  --no-api --sessions 1048576 --steps 5 --warmup 1 > $OUT/prof.log 2>&1 || exit $?
f=$(find $OUT/prof -name "*kernel_stats.csv" | head -1); cp "$f" $OUT/kernel_stats_r0.csv
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof1 -o run --output-format csv -- python bench.py --mix hetero --no-scalar \
  --no-api --sessions 1048576 --steps 5 --warmup 1 > $OUT/prof1.log 2>&1 || exit $?
f=$(find $OUT/prof1 -name "*kernel_stats.csv" | head -1); cp "$f" $OUT/kernel_stats_r1.csv
