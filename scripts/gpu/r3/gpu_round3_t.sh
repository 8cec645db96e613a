#!/bin/bash
# PMC passes over the hetero-mix batch kernels (counters only; one pass per counter group).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp AHV_SKIP_AUTOBUILD=1
OUT=gpurun_out/r3t
mkdir -p $OUT
run() {  # $1 name, $2 counters
  timeout -s KILL 120 rocprofv3 --pmc $2 --kernel-include-regex store_pipe --output-format csv -d $OUT/$1 -o pmc -- python3 bench.py --mix hetero --sessions 262144 --steps 2 --warmup 1 --no-scalar --no-api --no-liability > $OUT/$1.log 2>&1 || return 1
  python3 scripts/pmc_summary.py $(find $OUT/$1 -name "*counter_collection.csv" | head -1) > $OUT/$1.md || return 1
}
run issue "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY" &&
run stall "SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_THREAD_CYCLES_VALU SQ_INSTS_VALU_INT" &&
run mem "TCC_HIT_sum TCC_MISS_sum" &&
echo done
