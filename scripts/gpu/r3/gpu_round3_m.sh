#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp AHV_SKIP_AUTOBUILD=1
OUT=gpurun_out/r3m
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_reference_trace.py tests/test_api_concurrency.py tests/test_saga_runner.py tests/test_store.py tests/test_device_engines.py > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
timeout -k 10 300 python -u benchmarks/bench_engines.py > $OUT/engines.log 2>&1 || exit 1
for i in 1 2 3; do
  AHV_STEP_SPECULATE=1 timeout -k 10 120 python -u scripts/p50_ab.py 2000 >> $OUT/p50_spec.jsonl 2>/dev/null || exit 1
  AHV_STEP_SPECULATE=0 timeout -k 10 120 python -u scripts/p50_ab.py 2000 >> $OUT/p50_nospec.jsonl 2>/dev/null || exit 1
done
echo done
