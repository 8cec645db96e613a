#!/bin/bash
# Round 5, call aj: lane orders from one packed-key argsort — batched API GPU tests and
# the hetero batch end to end.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp AHV_SKIP_AUTOBUILD=1
OUT=gpurun_out/r5aj
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_store_pipeline.py tests/test_gpu_pipeline.py -m gpu -x -q -p no:cacheprovider \
  --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1; rc=$?
tail -2 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python benchmarks/bench_api.py --n 0 --batch 20000 --rounds 7 > $OUT/api.json 2>&1 || exit $?
grep -v amdgpu $OUT/api.json | tail -1 | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print({k: (d[k]["sessions_per_s"], d[k]["phases_ms"]) for k in ("batch", "batch_hetero")})'
