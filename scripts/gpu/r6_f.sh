#!/bin/bash
# Round 6, call f: speculated chain links — the host prefills its predicted parent
# digest; two helper waves hash whole records off the chain, the engine checks the
# parent and takes the digest.  Worker tests, root stress, per-call timeline, split.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp AHV_SKIP_AUTOBUILD=1 AHV_SPEC_TERMINATE=0
OUT=gpurun_out/r6f
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_reference_trace.py tests/test_speculation.py tests/test_gpu_store.py \
  tests/test_api_concurrency.py tests/test_store_fuzz.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1; rc=$?
tail -2 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python scripts/root_stress.py 6000 cuda > $OUT/stress.txt 2>&1 || exit $?
tail -1 $OUT/stress.txt | cut -c1-200
timeout -k 10 200 python scripts/percall_timeline.py > $OUT/timeline.jsonl 2>&1 || exit $?
grep -E "p50|CAPTURE|CLOSE" $OUT/timeline.jsonl | cut -c1-330
timeout -k 10 200 python scripts/percall_split.py cuda > $OUT/split.txt 2>&1 || exit $?
grep -v amdgpu $OUT/split.txt | tail -11
AHV_STORE_SPEC_CHAIN=0 timeout -k 10 200 python scripts/percall_split.py cuda > $OUT/split_nospec.txt 2>&1 || exit $?
grep -v amdgpu $OUT/split_nospec.txt | tail -1
timeout -k 10 300 python scripts/profile_gather.py > $OUT/gather.txt 2>&1 || exit $?
head -3 $OUT/gather.txt | cut -c1-400
