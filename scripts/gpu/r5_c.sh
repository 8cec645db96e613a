#!/bin/bash
# Round 5, call c: the whole -m gpu suite after the double-release fix, the bench
# (post-timing oracle check), and the per-call baseline with device-awaited terminate
# roots (AHV_SPEC_TERMINATE=0) next to the speculated one, plus gather at 10^4.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp AHV_SKIP_AUTOBUILD=1
OUT=gpurun_out/r5c
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread \
  > $OUT/pytest.log 2>&1; echo tests rc=$?
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > $OUT/bench.log 2>&1 && echo bench-ok && \
AHV_SPEC_TERMINATE=0 ITERS=3000 timeout -k 10 300 python scripts/profile_percall.py > $OUT/percall_awaited.log 2>&1 && \
ITERS=3000 timeout -k 10 300 python scripts/profile_percall.py > $OUT/percall_spec.log 2>&1 && \
AHV_SPEC_TERMINATE=0 N=10000 timeout -k 10 300 python scripts/profile_gather.py > $OUT/gather_awaited.log 2>&1 && \
timeout -k 10 300 python scripts/percall_split.py cuda > $OUT/split_cuda.txt 2>&1; echo profiles rc=$?
tail -1 $OUT/pytest.log
tail -1 $OUT/bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print({k: d.get(k) for k in ('value','ms_per_step','headline_verified','headline_verified_sessions','headline_kernel','device_p50_us','device_mean_us','scalar_p50_us','api_gather_pipelines_per_s')})"
grep p50_us $OUT/percall_awaited.log | cut -c1-300; grep p50_us $OUT/percall_spec.log | cut -c1-300
head -3 $OUT/gather_awaited.log | cut -c1-250; cat $OUT/split_cuda.txt | grep -v amdgpu
