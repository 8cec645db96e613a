#!/bin/bash
# Round 4, call ai: VALU issue of the headline kernel (store_template_kernel<3,3>) at
# 1 M sessions per step — how close the SHA-bound kernel is to the VALU issue limit.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp AHV_SKIP_AUTOBUILD=1
OUT=gpurun_out/r4ai
mkdir -p $OUT
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY \
  --kernel-include-regex store_template --output-format csv -d $OUT/pmc -o pmc -- \
  python3 bench.py --steps 2 --warmup 1 --no-scalar --no-api --sessions 1048576 > $OUT/pmc.log 2>&1 && echo pmc-ok && \
python scripts/pmc_summary.py $(find $OUT/pmc -name "*counter_collection.csv" | head -1) > $OUT/pmc.md && \
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/kt -o kt -- python3 bench.py --steps 4 --warmup 1 --no-scalar --no-api --sessions 1048576 > $OUT/kt.log 2>&1 && echo kt-ok && \
python scripts/prof_summary.py $(find $OUT/kt -name "*.db" | head -1) > $OUT/kt.md
rc=$?
rm -rf $OUT/pmc $OUT/kt
cat $OUT/pmc.md | cut -c1-300
head -6 $OUT/kt.md | cut -c1-200
exit $rc
