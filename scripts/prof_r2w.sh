#!/bin/bash
# GPU tests, headline bench, config4 (coroutine sagas through the device FSM).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp AHV_SKIP_AUTOBUILD=1
OUT=gpurun_out/r2w
mkdir -p $OUT
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 &&
timeout -k 10 300 python3 bench.py > $OUT/bench.log 2>&1 &&
timeout -k 10 300 python3 benchmarks/bench_configs.py config4 > $OUT/config4.log 2>&1
