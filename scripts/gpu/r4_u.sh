#!/bin/bash
# Round 4, call u: one fence per post (sequence chunk written last), posts write only the slot
# words in use — store/API GPU tests, call probe, per-call split, p50 and gather.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp AHV_SKIP_AUTOBUILD=1
OUT=gpurun_out/r4u
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_store.py tests/test_gpu_store.py tests/test_store_fuzz.py tests/test_api_concurrency.py \
  tests/test_speculation.py tests/test_reference_trace.py tests/test_checkpoint.py tests/test_device_engines.py -m gpu -x -q \
  -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 && echo tests-ok && \
timeout -k 10 300 python scripts/probe_calls.py > $OUT/probe_calls.log 2>&1 && echo probe-ok && \
timeout -k 10 300 python scripts/percall_split.py cuda > $OUT/split_cuda.txt 2>&1 && echo split-ok && \
ITERS=2000 timeout -k 10 300 python scripts/profile_percall.py > $OUT/percall.log 2>&1 && echo percall-ok && \
N=10000 timeout -k 10 300 python scripts/profile_gather.py > $OUT/gather.log 2>&1 && echo gather-ok && \
timeout -k 10 300 python scripts/probe_worker.py > $OUT/probe_worker.log 2>&1 && echo worker-ok
rc=$?
tail -1 $OUT/pytest.log; tail -1 $OUT/probe_calls.log; cat $OUT/split_cuda.txt
grep p50_us $OUT/percall.log | cut -c1-200; head -3 $OUT/gather.log | cut -c1-200; tail -1 $OUT/probe_worker.log
exit $rc
