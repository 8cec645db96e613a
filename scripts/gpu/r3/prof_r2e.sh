#!/bin/bash
# config5 (honest storm) + its traffic passes; slash/sigma stall split; merkle trace for the record.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp AHV_SKIP_AUTOBUILD=1
OUT=gpurun_out/r2e
mkdir -p $OUT
step() { echo "[prof_r2e] $(date +%T) $1"; }
pmc() {
  local name=$1 rx=$2 ctr=$3; shift 3
  step "pmc $name"
  timeout -s KILL 150 rocprofv3 --pmc $ctr --kernel-include-regex "$rx" --output-format csv -d $OUT/pmc_$name -o pmc -- "$@" \
    > $OUT/pmc_$name.log 2>&1
}
C5="python3 benchmarks/bench_configs.py config5 --steps 2 --warmup 1"
step tests && timeout -k 10 200 python3 -u -m pytest -m gpu -x -v --timeout 120 --timeout-method thread \
  tests/test_saga_runner.py tests/test_gpu_kernels.py > $OUT/tests.log 2>&1 &&
step config5 && timeout -k 10 300 python3 benchmarks/bench_configs.py config5 --steps 10 --warmup 2 > $OUT/config5.log 2>&1 &&
step config4 && timeout -k 10 300 python3 benchmarks/bench_configs.py config4 --steps 5 --warmup 1 > $OUT/config4.log 2>&1 &&
step trace5 && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace_c5 -o run -- $C5 > $OUT/trace_c5.log 2>&1 &&
pmc c5_fetch "chain_hash|merkle|slash|sigma_eff" "FETCH_SIZE GRBM_GUI_ACTIVE" $C5 &&
pmc c5_write "chain_hash|merkle|slash|sigma_eff" "WRITE_SIZE GRBM_GUI_ACTIVE" $C5 &&
pmc c5_stall "chain_hash|merkle|slash|sigma_eff" "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM SQ_INSTS_LDS SQ_WAVES" $C5
rc=$?
step "done rc=$rc"
exit $rc
