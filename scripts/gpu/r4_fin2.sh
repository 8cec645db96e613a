#!/bin/bash
# Round 4, call fin2: round-end rehearsal with light result publication, next-slot prefetch and narrowed FREE_ROWS drains on by default — full GPU suite, smoke,
# the default bench, configs 2/3 and the hetero line.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp AHV_SKIP_AUTOBUILD=1
OUT=gpurun_out/r4fin2
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread \
  > $OUT/pytest_gpu.log 2>&1 && echo tests-ok && \
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 && echo smoke-ok && \
timeout -k 10 600 python bench.py > $OUT/bench.log 2>&1 && echo bench-ok && \
timeout -k 10 300 python benchmarks/bench_configs.py config2 config3 config4 config5 > $OUT/configs.log 2>&1 && echo configs-ok && \
timeout -k 10 300 python bench.py --mix hetero --no-scalar --no-api --steps 20 --warmup 3 > $OUT/hetero.log 2>&1 && echo hetero-ok && \
ITERS=3000 timeout -k 10 300 python scripts/profile_percall.py > $OUT/percall.log 2>&1 && echo percall-ok && \
timeout -k 10 300 python scripts/percall_outliers.py cuda 5000 > $OUT/outliers.txt 2>&1 && echo outliers-ok
rc=$?
tail -3 $OUT/pytest_gpu.log; tail -2 $OUT/smoke.log
tail -1 $OUT/bench.log | cut -c1-700
cut -c1-250 $OUT/configs.log
tail -1 $OUT/hetero.log | cut -c1-250
sed -n 2,5p $OUT/outliers.txt | cut -c1-200
exit $rc
