#!/bin/bash
# Round 5, call o: more samples of the divergence stress per worker feature set.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp AHV_SKIP_AUTOBUILD=1
OUT=gpurun_out/r5o
mkdir -p $OUT
S="timeout -k 10 200 python scripts/root_stress.py 6000 cuda"
for k in 1 2; do
  AHV_STORE_SPECULATE=0 $S > $OUT/nospec$k.txt 2>&1 || exit $?; tail -1 $OUT/nospec$k.txt | cut -c1-200
  AHV_STORE_PREFIX=0 $S > $OUT/noprefix$k.txt 2>&1 || exit $?; tail -1 $OUT/noprefix$k.txt | cut -c1-200
done
$S > $OUT/default.txt 2>&1 || exit $?; tail -1 $OUT/default.txt | cut -c1-1500
