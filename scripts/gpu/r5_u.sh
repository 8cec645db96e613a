#!/bin/bash
# Round 5, call u: where the host CPU of the concurrent per-call path goes
# (device vs host engines, own and cumulative time).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp AHV_SKIP_AUTOBUILD=1
OUT=gpurun_out/r5u
mkdir -p $OUT
N=10000 TOP=45 timeout -k 10 300 python scripts/profile_gather.py > $OUT/gather_tot.txt 2>&1 || exit $?
N=10000 TOP=60 SORT=cumulative timeout -k 10 300 python scripts/profile_gather.py > $OUT/gather_cum.txt 2>&1 || exit $?
DEV=host N=10000 TOP=60 SORT=cumulative timeout -k 10 300 python scripts/profile_gather.py > $OUT/host_cum.txt 2>&1 || exit $?
grep -v amdgpu $OUT/gather_tot.txt | head -3; grep -v amdgpu $OUT/host_cum.txt | head -3
