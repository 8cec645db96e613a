#!/bin/bash
# Liability kernels round 3: new GPU tests, bench_liability variants, config5
# (split vs round-2 group pass), kernel trace of config5, stall counters.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp AHV_SKIP_AUTOBUILD=1
OUT=gpurun_out/r3e
mkdir -p $OUT
echo "[r3e] $(date +%T) tests"
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_kernels.py > $OUT/tests.log 2>&1 || { echo "tests failed"; tail -30 $OUT/tests.log; exit 1; }
echo "[r3e] $(date +%T) bench_liability"
timeout -k 10 300 python -u benchmarks/bench_liability.py --iters 30 > $OUT/liab.log 2>&1 || { tail -20 $OUT/liab.log; exit 1; }
echo "[r3e] $(date +%T) config5"
timeout -k 10 200 python -u benchmarks/bench_configs.py config5 --steps 10 --warmup 2 > $OUT/c5_split.log 2>&1 &&
AHV_SLASH_FUSED=1 timeout -k 10 200 python -u benchmarks/bench_configs.py config5 --steps 10 --warmup 2 > $OUT/c5_group.log 2>&1 &&
timeout -k 10 200 python -u benchmarks/bench_configs.py config5 --steps 10 --warmup 2 > $OUT/c5_split2.log 2>&1 || exit 1
echo "[r3e] $(date +%T) trace"
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_c5 -o c5 -- python3 benchmarks/bench_configs.py config5 --steps 10 --warmup 2 > $OUT/trace_c5.log 2>&1 || exit 1
RX="slash|sigma|exposure"
pmc() {
  local name=$1 ctr=$2
  echo "[r3e] $(date +%T) pmc $name"
  timeout -s KILL 150 rocprofv3 --pmc $ctr --kernel-include-regex "$RX" --output-format csv -d $OUT/pmc_$name -o pmc -- python3 benchmarks/bench_liability.py --iters 3 --sessions 1250000 --only exposure,stream,csr,slash_split,slash_group > $OUT/pmc_$name.log 2>&1
}
pmc stall "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM SQ_INSTS_LDS SQ_INSTS_SALU" &&
pmc fetch "FETCH_SIZE GRBM_GUI_ACTIVE"
echo "[r3e] $(date +%T) done"
