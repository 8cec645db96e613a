#!/bin/bash
# Liability A/B: LDS-staged cascade, stream-kernel slice counts, K03 form in the split slash.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp AHV_SKIP_AUTOBUILD=1
OUT=gpurun_out/r3f
mkdir -p $OUT
echo "[r3f] $(date +%T) tests"
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_kernels.py > $OUT/tests.log 2>&1 || { echo "tests failed"; tail -30 $OUT/tests.log; exit 1; }
for k in 1 2 4; do
  echo "[r3f] $(date +%T) slices $k"
  AHV_STREAM_SLICES=$k timeout -k 10 200 python -u benchmarks/bench_liability.py --iters 30 --only stream,csr,slash_split > $OUT/liab_k$k.log 2>&1 || exit 1
done
echo "[r3f] $(date +%T) config5"
for v in "AHV_STREAM_SLICES=1" "AHV_STREAM_SLICES=2" "AHV_SLASH_SIGMA=csr" "AHV_SLASH_FUSED=1" "AHV_STREAM_SLICES=1"; do
  env $v timeout -k 10 200 python -u benchmarks/bench_configs.py config5 --steps 10 --warmup 2 > $OUT/c5_$v.log 2>&1 || exit 1
  echo "$v $(grep -o '"ms_per_storm": [0-9.]*' $OUT/c5_$v.log)" >> $OUT/c5_summary.txt
done
echo "[r3f] $(date +%T) trace"
AHV_STREAM_SLICES=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_c5 -o c5 -- python3 benchmarks/bench_configs.py config5 --steps 10 --warmup 2 > $OUT/trace_c5.log 2>&1 || exit 1
echo "[r3f] $(date +%T) pmc"
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM SQ_INSTS_LDS SQ_INSTS_SALU --kernel-include-regex "slash|sigma|exposure" --output-format csv -d $OUT/pmc_stall -o pmc -- python3 benchmarks/bench_liability.py --iters 3 --sessions 1250000 --only exposure,stream,csr,slash_split > $OUT/pmc_stall.log 2>&1
echo "[r3f] $(date +%T) done"
