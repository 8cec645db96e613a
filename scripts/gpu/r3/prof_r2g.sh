#!/bin/bash
# Re-entry refresh: headline trace, configs 3/5 timings, config5 trace + stall split
# after the chain_hash prefetch emitter and the 64-lane store hash engine.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp AHV_SKIP_AUTOBUILD=1
OUT=gpurun_out/r2g
mkdir -p $OUT
step() { echo "[prof_r2g] $(date +%T) $1"; }
pmc() {
  local name=$1 rx=$2 ctr=$3; shift 3
  step "pmc $name"
  timeout -s KILL 150 rocprofv3 --pmc $ctr --kernel-include-regex "$rx" --output-format csv -d $OUT/pmc_$name -o pmc -- "$@" \
    > $OUT/pmc_$name.log 2>&1
}
C5="python3 benchmarks/bench_configs.py config5 --steps 2 --warmup 1"
step config3 && timeout -k 10 300 python3 benchmarks/bench_configs.py config3 --steps 10 --warmup 2 > $OUT/config3.log 2>&1 &&
step config5 && timeout -k 10 300 python3 benchmarks/bench_configs.py config5 --steps 10 --warmup 2 > $OUT/config5.log 2>&1 &&
step trace_bench && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace_bench -o run -- python3 bench.py --steps 10 --warmup 2 --no-scalar > $OUT/trace_bench.log 2>&1 &&
step trace5 && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace_c5 -o run -- $C5 > $OUT/trace_c5.log 2>&1 &&
pmc c5_stall "chain_hash|merkle|slash|sigma_eff" "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM SQ_INSTS_LDS SQ_WAVES" $C5
rc=$?
step "done rc=$rc"
exit $rc
