#!/bin/bash
# Round 6, call u: ring lookahead (helper waves hash captures from the command ring
# ahead of the command wave, feature 256) — store GPU tests, root stress (device
# roots and digests vs hashlib), per-call timeline / split / p50 with it on and off.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp AHV_SKIP_AUTOBUILD=1
OUT=gpurun_out/r6u
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_speculation.py tests/test_gpu_store.py tests/test_store.py -m gpu -x -q -p no:cacheprovider --timeout 240 --timeout-method thread > $OUT/tests.txt 2>&1; rc=$?
tail -2 $OUT/tests.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python scripts/root_stress.py 6000 cuda > $OUT/root_stress.txt 2>&1 || exit $?
cat $OUT/root_stress.txt | tail -1 | cut -c1-200
for la in 1 0; do
  AHV_STORE_LOOKAHEAD=$la ITERS=400 timeout -k 10 200 python scripts/percall_timeline.py > $OUT/timeline_la$la.jsonl 2>&1 || exit $?
  AHV_STORE_LOOKAHEAD=$la ITERS=2000 timeout -k 10 200 python scripts/profile_percall.py > $OUT/percall_la$la.txt 2>&1 || exit $?
  AHV_STORE_LOOKAHEAD=$la N=10000 timeout -k 10 200 python scripts/profile_gather.py > $OUT/gather_la$la.txt 2>&1 || exit $?
  echo "lookahead=$la $(head -2 $OUT/percall_la$la.txt | tail -1 | cut -c1-120)"
  head -3 $OUT/gather_la$la.txt | grep pipelines_per_s | cut -c1-200
done
grep -v amdgpu $OUT/timeline_la1.jsonl | cut -c1-420
