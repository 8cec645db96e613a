#!/bin/bash
# Round 5, call r: headline kernel with the next delta's rows prefetched before the record
# stores and the block-0 copies deferred to one point — oracle tests, then the bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp AHV_SKIP_AUTOBUILD=1
OUT=gpurun_out/r5r
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_store_template.py tests/test_gpu_headline_oracle.py -m gpu -x -q \
  -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/oracle_tests.log 2>&1; rc=$?
tail -2 $OUT/oracle_tests.log; [ $rc -eq 0 ] || exit $rc
B="python bench.py --steps 10 --warmup 2 --no-scalar --no-api --no-liability --verify-sessions 64"
for k in 1 2; do
  timeout -k 10 300 $B > $OUT/base$k.log 2>&1 || exit $?
  echo "run$k $(tail -1 $OUT/base$k.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["headline_verified"])')"
done
