#!/bin/bash
# Round 4, call e: GPU suite + smoke on the store-backed engine, then the headline
# bench with both template-kernel occupancy variants, the graph bench, and a
# kernel-trace profile of the headline step.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp AHV_SKIP_AUTOBUILD=1
OUT=gpurun_out/r4e
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread \
  > $OUT/pytest_gpu.log 2>&1 && echo tests-ok && \
timeout -k 10 300 python __graft_entry__.py smoke > $OUT/smoke.log 2>&1 && echo smoke-ok && \
timeout -k 10 600 python bench.py --steps 20 --warmup 3 --scalar-iters 1000 > $OUT/bench.log 2>&1 && echo bench-ok && \
AHV_TEMPLATE_WAVES=2 timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-scalar --no-api > $OUT/bench_w2.log 2>&1 && echo w2-ok && \
timeout -k 10 300 python bench.py --graph --steps 10 --warmup 2 --no-scalar --no-api > $OUT/bench_graph.log 2>&1 && echo graph-ok && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run -- python bench.py --steps 10 --warmup 2 --no-scalar --no-api > $OUT/prof.log 2>&1 && echo prof-ok
rc=$?
tail -5 $OUT/pytest_gpu.log; tail -2 $OUT/smoke.log; for f in bench bench_w2 bench_graph; do tail -1 $OUT/$f.log | cut -c1-300; done
exit $rc
