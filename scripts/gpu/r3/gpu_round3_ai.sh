#!/bin/bash
# Creation-stamp guard + deferred create: GPU tests, p50 x3, breakdown, gather.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp AHV_SKIP_AUTOBUILD=1
OUT=gpurun_out/r3ai
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_speculation.py tests/test_reference_trace.py tests/test_api_concurrency.py tests/test_gpu_store.py tests/test_store_fuzz.py tests/test_store_lifecycle.py tests/test_runtime_knobs.py tests/test_gpu_capacity.py > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
for i in 1 2 3; do timeout -k 10 120 python -u scripts/p50_ab.py 2000 >> $OUT/p50.jsonl 2>/dev/null || exit 1; done
timeout -k 10 120 python3 scripts/store_probe.py cuda 1000 breakdown > $OUT/breakdown_cuda.json 2> $OUT/err.log || exit 1
timeout -k 10 200 python -u -c "
import sys, json; sys.path.insert(0, '.'); sys.path.insert(0, 'benchmarks')
from bench_api import api_throughput
print(json.dumps(api_throughput('cuda', 10000, rounds=3)))" > $OUT/gather.json 2>> $OUT/err.log || exit 1
echo done
