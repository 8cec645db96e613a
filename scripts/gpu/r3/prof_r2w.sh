#!/bin/bash
# Closing run of the session: GPU tests, headline bench (default and --no-liability),
# BASELINE configs 2-5, headline kernel trace.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp AHV_SKIP_AUTOBUILD=1
OUT=gpurun_out/r2w
mkdir -p $OUT
step() { echo "[prof_r2w] $(date +%T) $1"; }
step tests && timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 &&
step smoke && timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 &&
step bench && timeout -k 10 300 python3 bench.py > $OUT/bench.log 2>&1 &&
step bench_noliab && timeout -k 10 120 python3 bench.py --no-scalar --no-liability > $OUT/bench_noliab.log 2>&1 &&
step configs && timeout -k 10 300 python3 benchmarks/bench_configs.py > $OUT/configs.log 2>&1 &&
step trace && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_bench -o run -- python3 bench.py --steps 10 --warmup 2 --no-scalar > $OUT/trace_bench.log 2>&1
rc=$?
step "done rc=$rc"
exit $rc
