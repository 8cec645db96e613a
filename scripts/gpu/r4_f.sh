#!/bin/bash
# Round 4, call f: GPU suite after the columnar checkpoint / sharded changes, and the
# columnar checkpoint at 10^5 and 10^6 sessions on the device store.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp AHV_SKIP_AUTOBUILD=1
OUT=gpurun_out/r4f
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread \
  > $OUT/pytest_gpu.log 2>&1 && echo tests-ok && \
timeout -k 10 300 python benchmarks/bench_checkpoint.py --sessions 100000 --device cuda > $OUT/ck_100k.log 2>&1 && echo ck100k-ok && \
timeout -k 10 600 python benchmarks/bench_checkpoint.py --sessions 1000000 --device cuda --dir /tmp/ahvck > $OUT/ck_1m.log 2>&1 && echo ck1m-ok && \
ITERS=2000 timeout -k 10 300 python scripts/profile_percall.py > $OUT/percall.log 2>&1 && echo percall-ok && \
timeout -k 10 300 python benchmarks/bench_mfma_ab.py > $OUT/mfma_ab.log 2>&1 && echo mfma-ab-ok
rc=$?
tail -3 $OUT/pytest_gpu.log; tail -1 $OUT/ck_100k.log; tail -1 $OUT/ck_1m.log; head -1 $OUT/percall.log; cat $OUT/mfma_ab.log
exit $rc
