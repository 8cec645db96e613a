#!/bin/bash
# Round 5, call h: pre-rendered changes fragments in the headline kernel (scalar-cache
# copies instead of per-pass string-pool reads) — oracle tests, then bench A/B.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp AHV_SKIP_AUTOBUILD=1
OUT=gpurun_out/r5h
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_store_template.py tests/test_gpu_headline_oracle.py -m gpu -x -q \
  -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/oracle_tests.log 2>&1; rc=$?
tail -3 $OUT/oracle_tests.log; [ $rc -eq 0 ] || exit $rc
B="python bench.py --steps 10 --warmup 2 --no-scalar --no-api --no-liability --verify-sessions 0"
for cfg in "1 0" "0 0" "1 12" "0 12"; do
  set -- $cfg
  AHV_TEMPLATE_FRAG=$1 AHV_TEMPLATE_AB=$2 timeout -k 10 300 $B > $OUT/frag$1_ab$2.log 2>&1 || exit $?
  echo "frag=$1 ab=$2 $(tail -1 $OUT/frag$1_ab$2.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-scalar --no-api > $OUT/bench_full.log 2>&1; rc=$?
tail -1 $OUT/bench_full.log | cut -c1-400
exit $rc
