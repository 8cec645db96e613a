#!/bin/bash
# Round 5, call e: worker timeline with the engine's stage / hash split and the
# command wave's prefix blocks; the batched-API phases (hetero and template) at 2·10⁴.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp AHV_SKIP_AUTOBUILD=1
OUT=gpurun_out/r5e
mkdir -p $OUT
# the worker changed (engine chain cache): its oracle tests first
timeout -k 10 400 python -u -m pytest tests/test_reference_trace.py tests/test_speculation.py tests/test_gpu_store.py -m gpu -x -q \
  -p no:cacheprovider --timeout 240 --timeout-method thread > $OUT/worker_tests.log 2>&1; rc=$?
tail -3 $OUT/worker_tests.log; [ $rc -eq 0 ] || exit $rc
AHV_SPEC_TERMINATE=0 timeout -k 10 300 python scripts/percall_timeline.py > $OUT/timeline_awaited.jsonl 2>&1 && \
timeout -k 10 300 python benchmarks/bench_api.py --device cuda --n 200 --batch 20000 --rounds 5 > $OUT/api.json 2>&1
rc=$?
[ $rc -eq 0 ] || exit $rc
# headline kernel attribution: 0 full, 4 no Merkle, 8 no record SHA, 12 neither (emission + rows + tee)
B="python bench.py --steps 5 --warmup 1 --no-scalar --no-api --no-liability --verify-sessions 0"
for ab in 0 4 8 12; do
  AHV_TEMPLATE_AB=$ab timeout -k 10 300 $B > $OUT/ab_$ab.log 2>&1 || exit $?
  echo "ab=$ab $(tail -1 $OUT/ab_$ab.log | cut -c1-160)"
done
# Merkle node pairing (ILP 2): <2,3,pair> and <3,3,pair> vs the default <3,3>
for w in 12 13 2; do
  AHV_TEMPLATE_WAVES=$w timeout -k 10 300 $B > $OUT/waves_$w.log 2>&1 || exit $?
  echo "waves=$w $(tail -1 $OUT/waves_$w.log | cut -c1-160)"
done
grep -v amdgpu $OUT/timeline_awaited.jsonl; tail -1 $OUT/api.json
exit $rc
