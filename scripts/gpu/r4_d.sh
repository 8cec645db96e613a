#!/bin/bash
# Round 4, call d: the whole GPU suite + smoke after moving the batched engine onto
# store rows (template kernel, ring mode, events, cursor), then the headline bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp AHV_SKIP_AUTOBUILD=1
OUT=gpurun_out/r4d
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread \
  > $OUT/pytest_gpu.log 2>&1 && echo tests-ok && \
timeout -k 10 300 python __graft_entry__.py smoke > $OUT/smoke.log 2>&1 && echo smoke-ok && \
timeout -k 10 600 python bench.py --steps 20 --warmup 3 --scalar-iters 1000 > $OUT/bench.log 2>&1 && echo bench-ok && \
timeout -k 10 300 python bench.py --graph --steps 10 --warmup 2 --no-scalar --no-api > $OUT/bench_graph.log 2>&1 && echo graph-ok
rc=$?
tail -5 $OUT/pytest_gpu.log; tail -2 $OUT/smoke.log; tail -1 $OUT/bench.log | cut -c1-400; tail -1 $OUT/bench_graph.log | cut -c1-300
exit $rc
