#!/bin/bash
# Round 6, call ao: the chain kernel's Merkle node through one compression site (chain
# kernel 156 -> 113 VGPRs: 4 waves per SIMD instead of 3) vs the K09 kernel — measured slower
# (chain 637 vs 611 us: the looped node loses the constant-folded padding block); reverted.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp AHV_SKIP_AUTOBUILD=1
OUT=gpurun_out/r6ao
mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests/test_store_pipeline.py tests/test_gpu_pipeline.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/tests.txt 2>&1; rc=$?
tail -2 $OUT/tests.txt; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for cr in 1 0; do
    for S in 1048576 4194304; do
      AHV_SP_CHAIN_ROOTS=$cr timeout -k 10 300 python bench.py --mix hetero --no-scalar --no-api --sessions $S --steps 20 --warmup 3 \
        > $OUT/h_r${cr}_${S}_$rep.json 2>$OUT/h_r${cr}_${S}_$rep.err || exit $?
      echo "rep=$rep chain_roots=$cr S=$S $(tail -1 $OUT/h_r${cr}_${S}_$rep.json | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
    done
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python bench.py --mix hetero \
  --no-scalar --no-api --sessions 1048576 --steps 5 --warmup 1 > $OUT/prof.log 2>&1 || exit $?
f=$(find $OUT/prof -name "*kernel_stats.csv" | head -1); cp "$f" $OUT/kernel_stats.csv
