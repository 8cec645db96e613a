#!/bin/bash
# Round-2 closing measurements: GPU tests, headline bench, configs 3-5, liability
# variants, hash-engine telemetry, kernel traces and a stall-counter pass.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp AHV_SKIP_AUTOBUILD=1
OUT=gpurun_out/r2n
mkdir -p $OUT
step() { echo "[prof_r2n] $(date +%T) $1"; }
pmc() {
  local name=$1 rx=$2 ctr=$3; shift 3
  step "pmc $name"
  timeout -s KILL 150 rocprofv3 --pmc $ctr --kernel-include-regex "$rx" --output-format csv -d $OUT/pmc_$name -o pmc -- "$@" \
    > $OUT/pmc_$name.log 2>&1
}
C5="python3 benchmarks/bench_configs.py config5 --steps 2 --warmup 1"
step tests && timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 &&
step bench && timeout -k 10 300 python3 bench.py > $OUT/bench.log 2>&1 &&
step bench_noliab && timeout -k 10 120 python3 bench.py --no-scalar --no-liability > $OUT/bench_noliab.log 2>&1 &&
step configs && timeout -k 10 300 python3 benchmarks/bench_configs.py > $OUT/configs.log 2>&1 &&
step liability && timeout -k 10 200 python3 benchmarks/bench_liability.py > $OUT/liability.log 2>&1 &&
step engine && timeout -k 10 100 python3 scripts/hash_engine_probe2.py cuda > $OUT/engine.log 2>&1 &&
step breakdown && timeout -k 10 100 python3 scripts/store_probe.py cuda 1000 breakdown > $OUT/breakdown.log 2>&1 &&
step trace_bench && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace_bench -o run -- python3 bench.py --steps 10 --warmup 2 --no-scalar > $OUT/trace_bench.log 2>&1 &&
step trace5 && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace_c5 -o run -- $C5 > $OUT/trace_c5.log 2>&1 &&
pmc c5_stall "chain_hash|merkle|slash|sigma_eff" "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM SQ_INSTS_LDS SQ_WAVES" $C5 &&
pmc c5_fetch "chain_hash|merkle|slash|sigma_eff" "FETCH_SIZE GRBM_GUI_ACTIVE" $C5
rc=$?
step "done rc=$rc"
exit $rc
