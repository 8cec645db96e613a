#!/bin/bash
# Golden traces on gfx950 + device p50 after the per-call micro-optimisations (3 runs) + stage breakdown.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp AHV_SKIP_AUTOBUILD=1
OUT=gpurun_out/r3x
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_reference_trace.py tests/test_api_concurrency.py tests/test_store.py > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
for i in 1 2 3; do timeout -k 10 120 python -u scripts/p50_ab.py 2000 >> $OUT/p50.jsonl 2>/dev/null || exit 1; done
timeout -k 10 120 python3 scripts/store_probe.py cuda 1000 breakdown > $OUT/breakdown_cuda.json 2> $OUT/err.log || exit 1
echo done
