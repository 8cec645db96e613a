#!/bin/bash
# Lifecycle speculation on gfx950: tests, p50 and gather A/B (AHV_SPEC_LIFECYCLE=1/0), stage breakdown.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp AHV_SKIP_AUTOBUILD=1
OUT=gpurun_out/r3af
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_speculation.py tests/test_reference_trace.py tests/test_api_concurrency.py tests/test_gpu_store.py tests/test_store_fuzz.py tests/test_saga_runner.py tests/test_store_lifecycle.py > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
for v in 1 0 1 0; do
  AHV_SPEC_LIFECYCLE=$v timeout -k 10 120 python -u scripts/p50_ab.py 2000 | sed "s/^{/{\"spec\": $v, /" >> $OUT/p50.jsonl || exit 1
done
for v in 1 0; do
  AHV_SPEC_LIFECYCLE=$v timeout -k 10 200 python -u -c "
import sys, json; sys.path.insert(0, '.'); sys.path.insert(0, 'benchmarks')
from bench_api import api_throughput
print(json.dumps(dict(spec=$v, **api_throughput('cuda', 10000, rounds=3))))" >> $OUT/gather.jsonl 2> $OUT/err.log || exit 1
done
timeout -k 10 120 python3 scripts/store_probe.py cuda 1000 breakdown > $OUT/breakdown_cuda.json 2>> $OUT/err.log || exit 1
echo done
