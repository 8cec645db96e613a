#!/bin/bash
# Round 5, call y: parallel merge of the spec walk — pack timings by thread count,
# the batched API tests, then the hetero batch end to end.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp AHV_SKIP_AUTOBUILD=1
OUT=gpurun_out/r5y
mkdir -p $OUT
AHV_PACK_DEBUG=1 timeout -k 10 300 python scripts/prof_prepare.py cuda > $OUT/prepare.txt 2>&1 || exit $?
grep -v amdgpu $OUT/prepare.txt | grep -v "^\[pack\]   part" | head -24
timeout -k 10 400 python -u -m pytest tests/test_store_pipeline.py -x -q -p no:cacheprovider --timeout 300 \
  --timeout-method thread > $OUT/tests.log 2>&1; rc=$?
tail -2 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python benchmarks/bench_api.py --n 0 --batch 20000 --rounds 5 > $OUT/api.json 2>&1 || exit $?
grep -v amdgpu $OUT/api.json | tail -1 | cut -c1-900
