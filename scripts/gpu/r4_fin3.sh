#!/bin/bash
# Round 4, call fin3: final rehearsal of the round-end tree — full GPU suite, smoke, default bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp AHV_SKIP_AUTOBUILD=1
OUT=gpurun_out/r4fin3
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread \
  > $OUT/pytest_gpu.log 2>&1 && echo tests-ok && \
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 && echo smoke-ok && \
timeout -k 10 600 python bench.py > $OUT/bench.log 2>&1 && echo bench-ok
rc=$?
tail -2 $OUT/pytest_gpu.log; tail -1 $OUT/smoke.log
tail -1 $OUT/bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print({k: d.get(k) for k in ('value','ms_per_step','device_p50_us','device_mean_us','scalar_p50_us','api_gather_pipelines_per_s')})"
exit $rc
