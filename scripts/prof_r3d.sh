#!/bin/bash
# Store worker: capture prefix cut short for a waiting command (per-block stop) —
# store GPU tests, then device p50 A/B (AHV_STORE_PREFIX_NOSTOP=1 restores the
# uninterrupted prefix), alternating, 3 runs each.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp AHV_SKIP_AUTOBUILD=1
OUT=gpurun_out/r3d
mkdir -p $OUT
P50="import bench, json; p, m = bench.scalar_pipeline_p50(2000, 'cuda'); print(json.dumps({'p50': round(p, 2), 'mean': round(m, 2)}))"
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_store.py tests/test_store_fuzz.py tests/test_reference_oracle.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || exit $?
for i in 1 2 3; do
  timeout -k 10 120 python3 -c "$P50" > $OUT/stop_$i.log 2>&1 || exit $?
  AHV_STORE_PREFIX_NOSTOP=1 timeout -k 10 120 python3 -c "$P50" > $OUT/nostop_$i.log 2>&1 || exit $?
done
