#!/bin/bash
# Round 5, call k: transposed (line-coalesced) record tee — oracle tests, then A/B vs the
# per-lane tee (AB 64), with and without SHA.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp AHV_SKIP_AUTOBUILD=1
OUT=gpurun_out/r5k
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_store_template.py tests/test_gpu_headline_oracle.py -m gpu -x -q \
  -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/oracle_tests.log 2>&1; rc=$?
tail -3 $OUT/oracle_tests.log; [ $rc -eq 0 ] || exit $rc
B="python bench.py --steps 10 --warmup 2 --no-scalar --no-api --no-liability --verify-sessions 0"
for ab in 0 64 12 76; do
  AHV_TEMPLATE_AB=$ab timeout -k 10 300 $B > $OUT/ab$ab.log 2>&1 || exit $?
  echo "ab$ab $(tail -1 $OUT/ab$ab.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
# per-call with the awaited default: split, gather (host CPU per pipeline)
timeout -k 10 300 python scripts/percall_split.py cuda > $OUT/split_awaited.txt 2>&1 || exit $?
grep -v amdgpu $OUT/split_awaited.txt | tail -12
N=10000 timeout -k 10 300 python scripts/profile_gather.py > $OUT/gather.txt 2>&1 || exit $?
grep -v amdgpu $OUT/gather.txt | tail -15
