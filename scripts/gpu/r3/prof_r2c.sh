#!/bin/bash
# GPU tests of the changed kernels, then the K03/K04 variant bench with HBM-traffic passes.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp AHV_SKIP_AUTOBUILD=1
OUT=gpurun_out/r2c
mkdir -p $OUT
step() { echo "[prof_r2c] $(date +%T) $1"; }
pmc() {
  local name=$1 rx=$2 ctr=$3; shift 3
  step "pmc $name"
  timeout -s KILL 120 rocprofv3 --pmc $ctr --kernel-include-regex "$rx" --output-format csv -d $OUT/pmc_$name -o pmc -- "$@" \
    > $OUT/pmc_$name.log 2>&1
}
LIAB="python3 benchmarks/bench_liability.py --iters 5"
step tests && timeout -k 10 400 python3 -u -m pytest -m gpu -x -v --timeout 120 --timeout-method thread \
  tests/test_gpu_kernels.py tests/test_gpu_pipeline.py tests/test_gpu_resources.py tests/test_device_engines.py \
  > $OUT/tests.log 2>&1 &&
step liability && timeout -k 10 200 python3 benchmarks/bench_liability.py > $OUT/liability.log 2>&1 &&
pmc liab_fetch "bond|build_tiles|sigma_eff" "FETCH_SIZE GRBM_GUI_ACTIVE" $LIAB &&
pmc liab_write "bond|build_tiles|sigma_eff" "WRITE_SIZE GRBM_GUI_ACTIVE" $LIAB &&
pmc liab_mix "bond|build_tiles|sigma_eff" "SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_VMEM SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAVES" $LIAB
rc=$?
step "done rc=$rc"
exit $rc
