#!/bin/bash
# Round 5, call ad: the lane renderer resolves a change's four strings (and their first chunks) before emitting them
# — batch tests, hetero bench, kernel stats.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp AHV_SKIP_AUTOBUILD=1
OUT=gpurun_out/r5ad
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_store_pipeline.py tests/test_gpu_pipeline.py -m gpu -x -q -p no:cacheprovider \
  --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1; rc=$?
tail -2 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  timeout -k 10 300 python bench.py --mix hetero --no-scalar --no-api --sessions 1048576 --steps 10 --warmup 2 \
    > $OUT/hetero$r.json 2>$OUT/hetero$r.err || exit $?
  tail -1 $OUT/hetero$r.json | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])'
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python bench.py --mix hetero --no-scalar \
  --no-api --sessions 1048576 --steps 5 --warmup 1 > $OUT/prof.log 2>&1 || exit $?
head -8 $OUT/prof/run_kernel_stats.csv | cut -c1-160
