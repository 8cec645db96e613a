#!/bin/bash
# Round 6, call aa: instruction-cache counters of the batched heterogeneous kernels
# (the render kernel is ~20 k instructions long after inlining).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp AHV_SKIP_AUTOBUILD=1
OUT=gpurun_out/r6aa
mkdir -p $OUT
B="python bench.py --mix hetero --sessions 1048576 --steps 2 --warmup 1 --no-scalar --no-api --no-liability --verify-sessions 0"
timeout -s KILL 120 rocprofv3 --pmc SQC_ICACHE_MISSES,SQC_ICACHE_HITS,SQ_WAVE_CYCLES,SQ_WAIT_INST_ANY -d $OUT/pmc_ic -o run --output-format csv -- $B > $OUT/pmc_ic.log 2>&1 || exit $?
echo "ic pass ok"
find $OUT -name "*counter_collection.csv" | head
