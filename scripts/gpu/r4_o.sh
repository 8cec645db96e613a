#!/bin/bash
# Round 4, call o: hetero A/B of the prefix-SHA placement (in the render pass vs its
# own kernel with lanes grouped by work, + K09 lanes by chain length), then the full
# GPU suite, smoke, configs 2/3, per-call + gather profiles and the default bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp AHV_SKIP_AUTOBUILD=1
OUT=gpurun_out/r4o
mkdir -p $OUT
B="python bench.py --mix hetero --no-scalar --no-api --steps 20 --warmup 3 --sessions 1048576"
timeout -k 10 300 $B > $OUT/h_render.log 2>&1 && echo h-render-ok && \
AHV_SP_PREFIX=sorted timeout -k 10 300 $B > $OUT/h_sorted.log 2>&1 && echo h-sorted-ok && \
AHV_SP_PREFIX=sorted AHV_SP_ORDER=5 timeout -k 10 300 $B > $OUT/h_sorted_k09.log 2>&1 && echo h-sorted-k09-ok && \
AHV_SP_PREFIX=kernel timeout -k 10 300 $B > $OUT/h_kernel.log 2>&1 && echo h-kernel-ok && \
AHV_SP_PREFIX=sorted AHV_SP_ORDER=5 timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_VALU SQ_THREAD_CYCLES_VALU SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_BUSY_CYCLES -d $OUT/ps -o pmc -- python3 bench.py --mix hetero --no-scalar --no-api --steps 3 --warmup 1 --sessions 262144 > $OUT/pmc_sorted.log 2>&1 && echo pmc-ok && \
python scripts/pmc_summary.py $(find $OUT/ps -name "*.db" | head -1) > $OUT/pmc_sorted.md
rc=$?
rm -rf $OUT/ps
for f in h_render h_sorted h_sorted_k09 h_kernel; do echo $f; tail -1 $OUT/$f.log | cut -c1-200; done
[ $rc -eq 0 ] && bash scripts/gpu/r4_n.sh
