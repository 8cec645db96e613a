#!/bin/bash
# Round-end rehearsal 3 (after the render-sink change), then PMC issue/stall passes over the batch kernels.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp AHV_SKIP_AUTOBUILD=1
OUT=gpurun_out/r3final3
mkdir -p $OUT
echo "[r3final3] $(date +%T) tests"
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ > $OUT/tests.log 2>&1 || { echo "tests failed"; tail -30 $OUT/tests.log; exit 1; }
echo "[r3final3] $(date +%T) smoke"
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
echo "[r3final3] $(date +%T) bench"
timeout -k 10 600 python -u bench.py > $OUT/bench.log 2>&1 || { tail -20 $OUT/bench.log; exit 1; }
run() {  # $1 name, $2 counters
  timeout -s KILL 120 rocprofv3 --pmc $2 --kernel-include-regex store_pipe --output-format csv -d $OUT/$1 -o pmc -- python3 bench.py --mix hetero --sessions 262144 --steps 2 --warmup 1 --no-scalar --no-api --no-liability > $OUT/$1.log 2>&1 || return 1
  python3 scripts/pmc_summary.py $(find $OUT/$1 -name "*counter_collection.csv" | head -1) > $OUT/$1.md || return 1
}
echo "[r3final3] $(date +%T) pmc"
run issue "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY" &&
run stall "SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_THREAD_CYCLES_VALU SQ_INSTS_VALU_INT" || exit 1
echo "[r3final3] $(date +%T) engines"
timeout -k 10 300 python -u benchmarks/bench_engines.py > $OUT/engines.log 2>&1 || exit 1 
echo "[r3final3] $(date +%T) configs"
timeout -k 10 600 python -u benchmarks/bench_configs.py config2 config3 config4 config5 > $OUT/configs.log 2>&1 || exit 1
echo "[r3final3] $(date +%T) done"
