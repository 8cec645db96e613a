#!/bin/bash
# Round 4, call m: the cooperative renderer (16/8/4 lanes per record, prefix SHA in
# its own kernel) vs the lane renderer — batch tests, hetero bench at 1M, a kernel
# trace and lane-utilisation PMC (summaries made here, databases removed).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp AHV_SKIP_AUTOBUILD=1
OUT=gpurun_out/r4m
mkdir -p $OUT
B="python bench.py --mix hetero --no-scalar --no-api --steps 20 --warmup 3 --sessions 1048576"
P="python3 bench.py --mix hetero --no-scalar --no-api --steps 3 --warmup 1 --sessions 262144"
C="SQ_INSTS_VALU SQ_THREAD_CYCLES_VALU SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_BUSY_CYCLES"
AHV_SP_RENDER=coop timeout -k 10 400 python -u -m pytest tests/test_store_pipeline.py -m gpu -x -q -p no:cacheprovider \
  --timeout 300 --timeout-method thread > $OUT/pytest_coop.log 2>&1 && echo tests-ok && \
AHV_SP_RENDER=coop AHV_SP_COOP_G=4 timeout -k 10 400 python -u -m pytest tests/test_store_pipeline.py -m gpu -x -q -p no:cacheprovider \
  --timeout 300 --timeout-method thread > $OUT/pytest_coop4.log 2>&1 && echo tests4-ok && \
timeout -k 10 300 $B > $OUT/h_lane.log 2>&1 && echo lane-ok && \
AHV_SP_RENDER=coop AHV_SP_COOP_G=16 timeout -k 10 300 $B > $OUT/h_c16.log 2>&1 && echo c16-ok && \
AHV_SP_RENDER=coop AHV_SP_COOP_G=8 timeout -k 10 300 $B > $OUT/h_c8.log 2>&1 && echo c8-ok && \
AHV_SP_RENDER=coop AHV_SP_COOP_G=4 timeout -k 10 300 $B > $OUT/h_c4.log 2>&1 && echo c4-ok && \
AHV_SP_RENDER=coop timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt -o kt -- python3 bench.py --mix hetero --no-scalar --no-api --steps 6 --warmup 2 --sessions 1048576 > $OUT/kt.log 2>&1 && echo kt-ok && \
python scripts/prof_summary.py $(find $OUT/kt -name "*.db" | head -1) > $OUT/kt_coop16.md && \
timeout -s KILL 200 rocprofv3 --pmc $C -d $OUT/pl -o pmc -- $P > $OUT/pmc_lane.log 2>&1 && echo pmc-lane-ok && \
python scripts/pmc_summary.py $(find $OUT/pl -name "*.db" | head -1) > $OUT/pmc_lane.md && \
AHV_SP_RENDER=coop timeout -s KILL 200 rocprofv3 --pmc $C -d $OUT/pc -o pmc -- $P > $OUT/pmc_coop.log 2>&1 && echo pmc-coop-ok && \
python scripts/pmc_summary.py $(find $OUT/pc -name "*.db" | head -1) > $OUT/pmc_coop16.md
rc=$?
rm -rf $OUT/kt $OUT/pl $OUT/pc
tail -1 $OUT/pytest_coop.log; tail -1 $OUT/pytest_coop4.log
for f in h_lane h_c16 h_c8 h_c4; do echo $f; tail -1 $OUT/$f.log | cut -c1-230; done
exit $rc
