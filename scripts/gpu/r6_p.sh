#!/bin/bash
# Round 6, call p: native per-call control plane (csrc/host/py_control.cpp) —
# GPU suite, per-call split and 10^4-concurrent gather with it on and off, host
# engines for comparison.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp AHV_SKIP_AUTOBUILD=1
OUT=gpurun_out/r6p
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/gpu_tests.txt 2>&1; rc=$?
tail -3 $OUT/gpu_tests.txt; [ $rc -eq 0 ] || exit $rc
for mode in 1 0; do
  AHV_NATIVE_CTL=$mode timeout -k 10 120 python scripts/percall_split.py cuda > $OUT/split_ctl$mode.txt 2>&1 || exit $?
  AHV_NATIVE_CTL=$mode N=10000 timeout -k 10 200 python scripts/profile_gather.py > $OUT/gather_ctl$mode.txt 2>&1 || exit $?
done
timeout -k 10 120 python scripts/percall_split.py host > $OUT/split_host.txt 2>&1 || exit $?
DEV=host N=10000 timeout -k 10 200 python scripts/profile_gather.py > $OUT/gather_host.txt 2>&1 || exit $?
AHV_NATIVE_CTL=1 ITERS=2000 timeout -k 10 200 python scripts/profile_percall.py > $OUT/percall_ctl1.txt 2>&1 || exit $?
for f in split_ctl1 split_ctl0 split_host; do echo "== $f"; cat $OUT/$f.txt | grep -v amdgpu.ids; done
for f in gather_ctl1 gather_ctl0 gather_host; do echo "== $f"; head -3 $OUT/$f.txt | grep pipelines_per_s | cut -c1-260; done
head -2 $OUT/percall_ctl1.txt | cut -c1-300
