#!/bin/bash
# Uniform-length K09 kernel: GPU tests for the audit kernels, then config5 A/B via traces.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp AHV_SKIP_AUTOBUILD=1
OUT=gpurun_out/r3a
mkdir -p $OUT
C5="python3 benchmarks/bench_configs.py config5 --steps 10 --warmup 2"
timeout -k 10 300 python3 -u -m pytest tests/test_merkle_tree.py tests/test_config5_arena.py tests/test_gpu_kernels.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 &&
timeout -k 10 200 $C5 > $OUT/c5.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- $C5 > $OUT/trace.log 2>&1
