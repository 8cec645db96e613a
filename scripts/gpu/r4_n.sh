#!/bin/bash
# Round 4, call n: full GPU suite on the current tree (small-batch template kernel,
# expectation queue, predicted terminates), smoke, configs 2/3, per-call + gather
# profiles and the default bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp AHV_SKIP_AUTOBUILD=1
OUT=gpurun_out/r4n
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread \
  > $OUT/pytest_gpu.log 2>&1 && echo tests-ok && \
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 && echo smoke-ok && \
timeout -k 10 300 python benchmarks/bench_configs.py config2 config3 > $OUT/configs.log 2>&1 && echo configs-ok && \
ITERS=2000 timeout -k 10 300 python scripts/profile_percall.py > $OUT/percall.log 2>&1 && echo percall-ok && \
N=10000 timeout -k 10 300 python scripts/profile_gather.py > $OUT/gather.log 2>&1 && echo gather-ok && \
timeout -k 10 600 python bench.py > $OUT/bench.log 2>&1 && echo bench-ok
rc=$?
tail -1 $OUT/pytest_gpu.log; tail -2 $OUT/smoke.log
cut -c1-300 $OUT/configs.log; grep p50_us $OUT/percall.log | cut -c1-220; head -3 $OUT/gather.log | cut -c1-250
tail -1 $OUT/bench.log | cut -c1-400
exit $rc
