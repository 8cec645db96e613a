#!/bin/bash
# Round 5, call n: which worker feature makes device roots diverge from the host's
# predictions?  The stress under the default and with the prefix wave / provisional
# trees / batched hashing switched off.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp AHV_SKIP_AUTOBUILD=1
OUT=gpurun_out/r5n
mkdir -p $OUT
S="timeout -k 10 200 python scripts/root_stress.py 6000 cuda"
$S > $OUT/default.txt 2>&1 || exit $?; tail -1 $OUT/default.txt
AHV_STORE_PREFIX=0 $S > $OUT/noprefix.txt 2>&1 || exit $?; tail -1 $OUT/noprefix.txt
AHV_STORE_SPECULATE=0 $S > $OUT/nospec.txt 2>&1 || exit $?; tail -1 $OUT/nospec.txt
AHV_STORE_BATCH=0 $S > $OUT/nobatch.txt 2>&1 || exit $?; tail -1 $OUT/nobatch.txt
