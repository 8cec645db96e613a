#!/bin/bash
# Round 5, call a: the production headline variants oracle-checked at 262,144 sessions
# (VERDICT r4 #2), the whole -m gpu suite, the bench with its post-timing oracle check,
# and the per-call baseline with device-awaited terminate roots (AHV_SPEC_TERMINATE=0).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp AHV_SKIP_AUTOBUILD=1
OUT=gpurun_out/r5a
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_headline_oracle.py -m gpu -x -v -p no:cacheprovider \
  --timeout 240 --timeout-method thread > $OUT/oracle.log 2>&1 && echo oracle-ok && \
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread \
  > $OUT/pytest.log 2>&1 && echo tests-ok && \
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > $OUT/bench.log 2>&1 && echo bench-ok && \
AHV_SPEC_TERMINATE=0 ITERS=3000 timeout -k 10 300 python scripts/profile_percall.py > $OUT/percall_awaited.log 2>&1 && echo percall-ok
rc=$?
tail -3 $OUT/oracle.log; tail -1 $OUT/pytest.log
tail -1 $OUT/bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print({k: d.get(k) for k in ('value','ms_per_step','headline_verified','headline_verified_sessions','headline_kernel','device_p50_us','device_mean_us','scalar_p50_us','api_gather_pipelines_per_s')})"
grep p50_us $OUT/percall_awaited.log | cut -c1-400
exit $rc
