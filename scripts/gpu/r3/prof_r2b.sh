#!/bin/bash
# Round-2 profiles of the new kernels (each GPU step under its own limit, && chained):
#   * K03/K04 variants: bench_liability (tiles pair vs CSR vs fused MFMA) + FETCH/WRITE/MFMA passes;
#   * K09 Merkle tree at 1e7 leaves: kernel trace + LDS bank-conflict pass;
#   * config3 with the fused liability stage.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp AHV_SKIP_AUTOBUILD=1
OUT=gpurun_out/r2b
mkdir -p $OUT
step() { echo "[prof_r2b] $(date +%T) $1"; }
pmc() {  # name, kernel regex, counters, command...
  local name=$1 rx=$2 ctr=$3; shift 3
  step "pmc $name"
  timeout -s KILL 120 rocprofv3 --pmc $ctr --kernel-include-regex "$rx" --output-format csv -d $OUT/pmc_$name -o pmc -- "$@" \
    > $OUT/pmc_$name.log 2>&1
}
LIAB="python3 benchmarks/bench_liability.py --iters 5"
step liability && timeout -k 10 200 python3 benchmarks/bench_liability.py > $OUT/liability.log 2>&1 &&
pmc liab_fetch "bond|build_tiles|sigma_eff" "FETCH_SIZE GRBM_GUI_ACTIVE" $LIAB &&
pmc liab_write "bond|build_tiles|sigma_eff" "WRITE_SIZE GRBM_GUI_ACTIVE" $LIAB &&
pmc liab_mix "bond|build_tiles|sigma_eff" "SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_VMEM SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAVES" $LIAB &&
step merkle-trace && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/trace_merkle -o run -- \
  python3 benchmarks/bench_merkle.py --sizes 10000000 --reps 3 --single-lane-max 0 > $OUT/trace_merkle.log 2>&1 &&
pmc merkle_lds merkle_tree "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAVES" \
  python3 benchmarks/bench_merkle.py --sizes 10000000 --reps 1 --single-lane-max 0 &&
step config3 && timeout -k 10 300 python3 benchmarks/bench_configs.py config3 --steps 10 --warmup 2 > $OUT/config3.log 2>&1 &&
timeout -k 10 300 python3 benchmarks/bench_configs.py config3 --tiles --steps 10 --warmup 2 >> $OUT/config3.log 2>&1
rc=$?
step "done rc=$rc"
exit $rc
