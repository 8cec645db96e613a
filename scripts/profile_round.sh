#!/bin/bash
# One GPU call that refreshes every profile summary committed under profiles/:
#   1. headline bench (1 GPU, with the scalar-API p50);
#   2. rocprofv3 kernel trace of the headline bench and of BASELINE configs 2-5;
#   3. counter passes (each its own run, --pmc only, no trace domains):
#        pipeline: VALU/SALU/LDS instruction mix + stall split;
#        pipeline: LDS bank conflicts + LDS activity;
#        configs:  fp64 MFMA ops (σ_eff bond tiles), LDS conflicts, VALU.
# Every GPU step runs under its own time limit; the first failure ends the call.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp AHV_SKIP_AUTOBUILD=1
OUT=gpurun_out/round
mkdir -p $OUT
step() { echo "[profile_round] $(date +%T) $1"; }
pmc() {  # name, kernel regex, counters, command...
  local name=$1 rx=$2 ctr=$3; shift 3
  step "pmc $name"
  timeout -s KILL 240 rocprofv3 --pmc $ctr --kernel-include-regex "$rx" --output-format csv -d $OUT/pmc_$name -o pmc -- "$@" \
    > $OUT/pmc_$name.log 2>&1
}
step bench && timeout -k 10 300 python3 bench.py --steps 20 --warmup 3 > $OUT/bench.log 2>&1 &&
step trace-bench && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace_bench -o run -- \
  python3 bench.py --steps 10 --warmup 2 --no-scalar > $OUT/trace_bench.log 2>&1 &&
step configs && timeout -k 10 400 python3 benchmarks/bench_configs.py --steps 10 --warmup 2 > $OUT/configs.log 2>&1 &&
step trace-configs && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/trace_configs -o run -- \
  python3 benchmarks/bench_configs.py --steps 5 --warmup 1 > $OUT/trace_configs.log 2>&1 &&
pmc pipe_mix governance "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
  python3 bench.py --steps 2 --warmup 1 --no-scalar &&
pmc pipe_lds governance "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU_INT32 SQ_INSTS_VMEM GRBM_GUI_ACTIVE" \
  python3 bench.py --steps 2 --warmup 1 --no-scalar &&
pmc cfg_mfma "bond_tiles|sigma_eff|slash|build_tiles|chain_hash|merkle|saga" \
  "SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVES" \
  python3 benchmarks/bench_configs.py --steps 2 --warmup 1 &&
pmc cfg_fetch "bond_tiles|sigma_eff|slash|build_tiles|chain_hash|merkle|saga" "FETCH_SIZE GRBM_GUI_ACTIVE" \
  python3 benchmarks/bench_configs.py --steps 2 --warmup 1 &&
pmc cfg_write "bond_tiles|sigma_eff|slash|build_tiles|chain_hash|merkle|saga" "WRITE_SIZE GRBM_GUI_ACTIVE" \
  python3 benchmarks/bench_configs.py --steps 2 --warmup 1 &&
pmc cfg_stall "slash|sigma_eff|build_tiles|chain_hash|merkle" "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES" \
  python3 benchmarks/bench_configs.py config5 config3 --steps 2 --warmup 1
rc=$?
step "done rc=$rc"
tail -1 $OUT/bench.log 2>/dev/null
exit $rc
