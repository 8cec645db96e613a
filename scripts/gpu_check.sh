#!/bin/bash
# One GPU session: GPU tests, smoke, short bench, rocprofv3 kernel stats.
# Every GPU step has its own time limit; steps are chained with && so the first
# failure (fault, abort, timeout) ends the call.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
export AHV_SKIP_AUTOBUILD=${AHV_SKIP_AUTOBUILD:-1}
OUT=gpurun_out
mkdir -p $OUT
STEPS=${STEPS:-all}
echo "[gpu_check] $(date) host=$(hostname) steps=$STEPS"
rocm-smi --showproductname > $OUT/rocm_smi.txt 2>&1 || true
run_tests() { timeout -k 10 600 python -m pytest tests -m gpu -q -p no:cacheprovider > $OUT/pytest_gpu.log 2>&1; }
run_smoke() { timeout -k 10 300 python __graft_entry__.py smoke > $OUT/smoke.log 2>&1; }
run_bench() { timeout -k 10 600 python bench.py --steps ${BENCH_STEPS:-10} --warmup 2 ${BENCH_ARGS:-} > $OUT/bench.log 2>&1; }
run_prof() {
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run -- python3 bench.py --steps 5 --warmup 1 --no-scalar ${BENCH_ARGS:-} > $OUT/prof.log 2>&1
}
case "$STEPS" in
  tests) run_tests ;;
  bench) run_bench ;;
  prof) run_prof ;;
  all) run_tests && echo tests-ok && run_smoke && echo smoke-ok && run_bench && echo bench-ok && run_prof && echo prof-ok ;;
  *) eval "$STEPS" ;;
esac
rc=$?
echo "[gpu_check] rc=$rc"
tail -5 $OUT/pytest_gpu.log 2>/dev/null; tail -3 $OUT/smoke.log 2>/dev/null; tail -2 $OUT/bench.log 2>/dev/null
exit $rc
