#!/bin/bash
# Round 4, call b: the store template pipeline on gfx950 — its tests, kernel
# resources, the headline bench over store rows, and a kernel-trace profile.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp AHV_SKIP_AUTOBUILD=1
OUT=gpurun_out/r4b
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_store_template.py tests/test_speculation.py -m gpu -x -q -p no:cacheprovider \
  --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 && echo tests-ok && \
timeout -k 10 120 python -c "
from agent_hypervisor_amd._native import C
for k in C.kernel_attributes():
    if 'template' in k['name'] or 'governance_pipeline' in k['name']: print(k)
" > $OUT/attrs.txt 2>&1 && \
timeout -k 10 600 python bench.py --steps 10 --warmup 2 --no-scalar --no-api > $OUT/bench.log 2>&1 && echo bench-ok && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run -- python3 bench.py --steps 5 --warmup 1 --no-scalar --no-api > $OUT/prof.log 2>&1 && echo prof-ok
rc=$?
tail -3 $OUT/pytest_gpu.log; cat $OUT/attrs.txt; tail -1 $OUT/bench.log | cut -c1-700
exit $rc
