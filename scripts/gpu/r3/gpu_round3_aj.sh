#!/bin/bash
# Capture prefix on the command wave even when the next command waits (AHV_STORE_PREFIX_ALWAYS) A/B.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp AHV_SKIP_AUTOBUILD=1
OUT=gpurun_out/r3aj
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_store.py tests/test_store_fuzz.py tests/test_reference_trace.py tests/test_speculation.py > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
for v in 1 0 1 0; do
  AHV_STORE_PREFIX_ALWAYS=$v timeout -k 10 120 python -u scripts/p50_ab.py 2000 | sed "s/^{/{\"always\": $v, /" >> $OUT/p50.jsonl || exit 1
  AHV_STORE_PREFIX_ALWAYS=$v timeout -k 10 120 python -u scripts/engine_probe.py 300 | sed "s/^{/{\"always\": $v, /" >> $OUT/engine.jsonl || exit 1
done
echo done
