#!/bin/bash
# Round 5, call p: the position-mixed slot checksum — divergence stress (several runs)
# and the new regression test.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp AHV_SKIP_AUTOBUILD=1
OUT=gpurun_out/r5p
mkdir -p $OUT
for k in 1 2 3; do
  timeout -k 10 200 python scripts/root_stress.py 6000 cuda > $OUT/stress$k.txt 2>&1 || exit $?
  tail -1 $OUT/stress$k.txt | cut -c1-300
done
timeout -k 10 400 python -u -m pytest tests/test_gpu_store.py tests/test_audit_verify.py tests/test_reference_trace.py -m gpu -x -q \
  -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1; rc=$?
tail -3 $OUT/tests.log
exit $rc
