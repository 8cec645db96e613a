#!/bin/bash
# Round 6, call au: chain lanes with each record's row fields loaded one record ahead vs in
# line — no gain (chain kernel 622 vs 613 us, step time equal: the lanes' waves already hide
# the row-field round trips); reverted, A/B kept in profiles/r6/hetero_chain_prefetch_ab_r6au.txt.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp AHV_SKIP_AUTOBUILD=1
OUT=gpurun_out/r6au
mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests/test_store_pipeline.py tests/test_gpu_pipeline.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/tests.txt 2>&1; rc=$?
tail -2 $OUT/tests.txt; [ $rc -eq 0 ] || exit $rc
for rep in 1 2 3; do
  for pf in 1 0; do
    AHV_SP_CHAIN_PREFETCH=$pf timeout -k 10 300 python bench.py --mix hetero --no-scalar --no-api --sessions 1048576 --steps 20 --warmup 3 \
      > $OUT/h_p${pf}_$rep.json 2>$OUT/h_p${pf}_$rep.err || exit $?
    echo "rep=$rep chain_prefetch=$pf $(tail -1 $OUT/h_p${pf}_$rep.json | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
for pf in 1 0; do
  AHV_SP_CHAIN_PREFETCH=$pf timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof$pf -o run --output-format csv -- python bench.py --mix hetero \
    --no-scalar --no-api --sessions 1048576 --steps 5 --warmup 1 > $OUT/prof$pf.log 2>&1 || exit $?
  f=$(find $OUT/prof$pf -name "*kernel_stats.csv" | head -1); cp "$f" $OUT/kernel_stats_p$pf.csv
done
