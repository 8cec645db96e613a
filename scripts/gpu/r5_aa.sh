#!/bin/bash
# Round 5, call aa: Merkle folded into the capture loop (D ≤ 3) —
# oracle tests, A/B of the occupancy variants, then the full default bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp AHV_SKIP_AUTOBUILD=1
OUT=gpurun_out/r5aa
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_store_template.py tests/test_gpu_headline_oracle.py -m gpu -x -q \
  -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/oracle_tests.log 2>&1; rc=$?
tail -3 $OUT/oracle_tests.log; [ $rc -eq 0 ] || exit $rc
B="python bench.py --steps 10 --warmup 2 --no-scalar --no-api --no-liability --verify-sessions 0"
for w in 3 2 3 2; do
  AHV_TEMPLATE_WAVES=$w timeout -k 10 300 $B > $OUT/w$w.log 2>&1 || exit $?
  echo "w$w $(tail -1 $OUT/w$w.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
timeout -k 10 600 python bench.py > $OUT/bench.json 2>$OUT/bench.err || exit $?
tail -1 $OUT/bench.json | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d.get("headline_verified"))'
