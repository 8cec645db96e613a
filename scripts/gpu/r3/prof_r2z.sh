#!/bin/bash
# Device single-session p50 after the terminate tweaks: store GPU tests, stage
# breakdown, p50 (3 runs of the reference harness through Hypervisor(device="cuda")).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp AHV_SKIP_AUTOBUILD=1
OUT=gpurun_out/r2z
mkdir -p $OUT
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_store.py tests/test_store_fuzz.py tests/test_reference_oracle.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 &&
timeout -k 10 120 python3 scripts/store_probe.py cuda 1000 breakdown > $OUT/breakdown.log 2>&1 &&
for i in 1 2 3; do timeout -k 10 120 python3 -c "
import bench, json
p, m = bench.scalar_pipeline_p50(2000, 'cuda')
print(json.dumps({'device_p50_us': round(p, 2), 'mean': round(m, 2)}))" > $OUT/p50_$i.log 2>&1 || exit $?; done
