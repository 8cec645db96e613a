#!/bin/bash
# Round 5, call q: the heterogeneous batched-API kernels as the timed step (1 M sessions),
# with a kernel trace for the per-kernel split.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp AHV_SKIP_AUTOBUILD=1
OUT=gpurun_out/r5q
mkdir -p $OUT
timeout -k 10 300 python bench.py --mix hetero --no-scalar --no-api --sessions 1048576 --steps 10 --warmup 2 \
  > $OUT/hetero.json 2>$OUT/hetero.err || exit $?
tail -1 $OUT/hetero.json | cut -c1-300
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run -- python bench.py --mix hetero --no-scalar \
  --no-api --sessions 1048576 --steps 5 --warmup 1 > $OUT/prof.log 2>&1 || exit $?
echo prof ok
