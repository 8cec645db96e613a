#!/bin/bash
# Round 4, call k: where the heterogeneous bench step and config2 spend their time
# (kernel traces with stats), and the plain hetero bench line.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp AHV_SKIP_AUTOBUILD=1
OUT=gpurun_out/r4k
mkdir -p $OUT
timeout -k 10 400 python bench.py --mix hetero --no-scalar --no-api --steps 20 --warmup 3 > $OUT/bench_hetero.log 2>&1 && echo hetero-ok && \
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/het -o het -- python3 bench.py --mix hetero --no-scalar --no-api --steps 10 --warmup 2 > $OUT/het_prof.log 2>&1 && echo het-prof-ok && \
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/c2 -o c2 -- python3 benchmarks/bench_configs.py config2 > $OUT/c2_prof.log 2>&1 && echo c2-prof-ok
rc=$?
tail -1 $OUT/bench_hetero.log | cut -c1-400
find $OUT -name "*kernel_stats.csv" | head
exit $rc
