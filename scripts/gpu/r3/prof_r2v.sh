#!/bin/bash
# K03/K04 fused MFMA kernel with zero-exposure atomics skipped: kernel tests,
# liability variants, config3.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp AHV_SKIP_AUTOBUILD=1
OUT=gpurun_out/r2v
mkdir -p $OUT
timeout -k 10 200 python3 -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 &&
timeout -k 10 200 python3 benchmarks/bench_liability.py > $OUT/liability.log 2>&1 &&
timeout -k 10 200 python3 benchmarks/bench_configs.py config3 > $OUT/config3.log 2>&1
