#!/bin/bash
# Round 6, call ak: cyclic-GC share of the 10^4-concurrent gather (scripts/probe_gc_gather.py)
# for gen-0 thresholds 5e4 (serving default), 2e5 and 1e6, device store and host engines.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp AHV_SKIP_AUTOBUILD=1
OUT=gpurun_out/r6ak
mkdir -p $OUT
for T in "50000,50,1000" "200000,20,1000" "1000000,10,1000"; do
  for D in cuda host; do
    AHV_GC_THRESHOLD=$T DEV=$D N=10000 timeout -k 10 200 python scripts/probe_gc_gather.py > $OUT/gc_${D}_${T%%,*}.jsonl 2> $OUT/gc_${D}_${T%%,*}.err || exit $?
    cut -c1-230 $OUT/gc_${D}_${T%%,*}.jsonl
  done
done
