#!/bin/bash
# Round 4, call a: the GPU suite after the native allocator / speculation-owner
# change, then the headline bench (short) for a baseline of this round.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp AHV_SKIP_AUTOBUILD=1
OUT=gpurun_out/r4a
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread \
  > $OUT/pytest_gpu.log 2>&1 && echo tests-ok && \
timeout -k 10 600 python bench.py --steps 10 --warmup 2 --scalar-iters 1000 > $OUT/bench.log 2>&1 && echo bench-ok
rc=$?
tail -5 $OUT/pytest_gpu.log; tail -1 $OUT/bench.log | cut -c1-1500
exit $rc
