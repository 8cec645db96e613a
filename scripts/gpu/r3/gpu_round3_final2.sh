#!/bin/bash
# Round-end rehearsal: every GPU test, smoke(), default bench.py (with the API section).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp AHV_SKIP_AUTOBUILD=1
OUT=gpurun_out/r3final2
mkdir -p $OUT
echo "[r3final2] $(date +%T) tests"
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ > $OUT/tests.log 2>&1 || { echo "tests failed"; tail -30 $OUT/tests.log; exit 1; }
echo "[r3final2] $(date +%T) smoke"
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
echo "[r3final2] $(date +%T) bench"
timeout -k 10 600 python -u bench.py > $OUT/bench.log 2>&1 || { tail -20 $OUT/bench.log; exit 1; }
echo "[r3final2] $(date +%T) engines"
timeout -k 10 300 python -u benchmarks/bench_engines.py > $OUT/engines.log 2>&1 || exit 1
echo "[r3final2] $(date +%T) configs"
timeout -k 10 600 python -u benchmarks/bench_configs.py config2 config3 config4 config5 > $OUT/configs.log 2>&1 || exit 1
echo "[r3final2] $(date +%T) done"
