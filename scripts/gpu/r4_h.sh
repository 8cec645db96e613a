#!/bin/bash
# Round 4, call h: command ring in pinned host memory (default) vs device memory
# with 32-byte BAR stores — post cost, per-call p50, the GPU suite, the full bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp AHV_SKIP_AUTOBUILD=1
OUT=gpurun_out/r4h
mkdir -p $OUT
timeout -k 10 300 python scripts/probe_worker.py > $OUT/probe_host.log 2>&1 && echo probe-host-ok && \
AHV_STORE_RING=device timeout -k 10 300 python scripts/probe_worker.py > $OUT/probe_dev.log 2>&1 && echo probe-dev-ok && \
ITERS=2000 timeout -k 10 300 python scripts/profile_percall.py > $OUT/percall_host.log 2>&1 && echo pc-host-ok && \
AHV_STORE_RING=device ITERS=2000 timeout -k 10 300 python scripts/profile_percall.py > $OUT/percall_dev.log 2>&1 && echo pc-dev-ok && \
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread \
  > $OUT/pytest_gpu.log 2>&1 && echo tests-ok && \
timeout -k 10 600 python bench.py --steps 20 --warmup 3 > $OUT/bench.log 2>&1 && echo bench-ok
rc=$?
tail -1 $OUT/probe_host.log; tail -1 $OUT/probe_dev.log; grep p50_us $OUT/percall_host.log | cut -c1-200; grep p50_us $OUT/percall_dev.log | cut -c1-200
tail -1 $OUT/pytest_gpu.log; tail -1 $OUT/bench.log | cut -c1-300
exit $rc
