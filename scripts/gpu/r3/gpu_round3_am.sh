#!/bin/bash
# Array-backed bulk row release/reclaim: store lifecycle GPU tests + batched API throughput.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp AHV_SKIP_AUTOBUILD=1
OUT=gpurun_out/r3am
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_store_lifecycle.py tests/test_store_pipeline.py tests/test_batched_views.py tests/test_gpu_store.py > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
timeout -k 10 300 python -u -c "
import sys, json; sys.path.insert(0, '.'); sys.path.insert(0, 'benchmarks')
from bench_api import batch_api_throughput
for _ in range(2):
    print(json.dumps(batch_api_throughput('cuda', 100000, 5)))
print(json.dumps(batch_api_throughput('cuda', 20000, 3, hetero=True)))" > $OUT/batch.jsonl 2> $OUT/err.log || exit 1
timeout -k 10 200 python -u scripts/batch_api_prof.py > $OUT/prof.log 2>&1 || exit 1
echo done
