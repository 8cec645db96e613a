#!/bin/bash
# Round 4, call t: with host-predicted terminates the hash engine's provisional
# Merkle roots are wasted work — A/B of AHV_STORE_SPECULATE (per-call p50/mean, gather).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp AHV_SKIP_AUTOBUILD=1
OUT=gpurun_out/r4t
mkdir -p $OUT
ITERS=3000 timeout -k 10 300 python scripts/profile_percall.py > $OUT/percall_on.log 2>&1 && echo on-ok && \
AHV_STORE_SPECULATE=0 ITERS=3000 timeout -k 10 300 python scripts/profile_percall.py > $OUT/percall_off.log 2>&1 && echo off-ok && \
N=10000 timeout -k 10 300 python scripts/profile_gather.py > $OUT/gather_on.log 2>&1 && echo gon-ok && \
AHV_STORE_SPECULATE=0 N=10000 timeout -k 10 300 python scripts/profile_gather.py > $OUT/gather_off.log 2>&1 && echo goff-ok && \
AHV_STORE_SPECULATE=0 timeout -k 10 300 python -u -m pytest tests/test_speculation.py tests/test_store.py -m gpu -x -q -p no:cacheprovider \
  --timeout 200 --timeout-method thread > $OUT/pytest_off.log 2>&1 && echo tests-off-ok
rc=$?
for f in percall_on percall_off; do grep p50_us $OUT/$f.log | cut -c1-230; done
for f in gather_on gather_off; do head -3 $OUT/$f.log | cut -c1-230; done
tail -1 $OUT/pytest_off.log
exit $rc
