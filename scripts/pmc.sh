#!/bin/bash
# Hardware-counter run of the pipeline kernel (counters only, no trace domains).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp AHV_SKIP_AUTOBUILD=1
mkdir -p gpurun_out
if [ "${LIST:-0}" = "1" ]; then timeout -k 10 120 rocprofv3 --list-avail > gpurun_out/counters.txt 2>&1; fi
PMC=${PMC:-"SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES"}
timeout -k 10 300 rocprofv3 --pmc $PMC --kernel-include-regex governance --output-format csv -d gpurun_out/pmc -o pmc -- python3 bench.py --steps 2 --warmup 1 --no-scalar --sessions ${SESS:-262144} > gpurun_out/pmc.log 2>&1
echo "rc=$?"
find gpurun_out/pmc -name "*.csv" | head
