#!/bin/bash
# Round 5, call b: diagnose the [cuda] template-batch participant mismatch seen after
# the 262,144-session oracle tests (r5a), then the two test files alone and in order.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp AHV_SKIP_AUTOBUILD=1
OUT=gpurun_out/r5b
mkdir -p $OUT
timeout -k 10 300 python -u scripts/gpu/r5_diag_template.py > $OUT/diag.log 2>&1; echo diag rc=$?
timeout -k 10 300 python -u -m pytest tests/test_store_template.py -m gpu -x -q -p no:cacheprovider --timeout 240 \
  --timeout-method thread > $OUT/alone.log 2>&1; echo alone rc=$?
timeout -k 10 300 python -u -m pytest tests/test_gpu_headline_oracle.py tests/test_store_template.py -m gpu -x -q \
  -p no:cacheprovider --timeout 240 --timeout-method thread > $OUT/pair.log 2>&1; echo pair rc=$?
cat $OUT/diag.log | grep -v amdgpu.ids; tail -2 $OUT/alone.log; tail -2 $OUT/pair.log
