#!/bin/bash
# Full GPU test suite, K03/K04 variants + traffic passes, config3/config4, headline bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp AHV_SKIP_AUTOBUILD=1
OUT=gpurun_out/r2d
mkdir -p $OUT
step() { echo "[prof_r2d] $(date +%T) $1"; }
pmc() {
  local name=$1 rx=$2 ctr=$3; shift 3
  step "pmc $name"
  timeout -s KILL 120 rocprofv3 --pmc $ctr --kernel-include-regex "$rx" --output-format csv -d $OUT/pmc_$name -o pmc -- "$@" \
    > $OUT/pmc_$name.log 2>&1
}
LIAB="python3 benchmarks/bench_liability.py --iters 5"
step tests && timeout -k 10 600 python3 -u -m pytest -m gpu -x -v --timeout 200 --timeout-method thread tests/ \
  > $OUT/tests.log 2>&1 &&
step liability && timeout -k 10 200 python3 benchmarks/bench_liability.py > $OUT/liability.log 2>&1 &&
pmc liab_fetch "bond|build_tiles|sigma_eff" "FETCH_SIZE GRBM_GUI_ACTIVE" $LIAB &&
pmc liab_write "bond|build_tiles|sigma_eff" "WRITE_SIZE GRBM_GUI_ACTIVE" $LIAB &&
pmc liab_mix "bond|build_tiles|sigma_eff" "SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_VMEM SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAVES" $LIAB &&
step configs && timeout -k 10 400 python3 benchmarks/bench_configs.py config3 config4 --steps 10 --warmup 2 > $OUT/configs.log 2>&1 &&
step bench && timeout -k 10 300 python3 bench.py > $OUT/bench.log 2>&1
rc=$?
step "done rc=$rc"
exit $rc
