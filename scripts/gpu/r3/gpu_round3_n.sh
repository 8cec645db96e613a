#!/bin/bash
# Device p50 stage breakdown: terminate with and without letting the hash engine drain first,
# and the host-engine breakdown on the same box for reference.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp AHV_SKIP_AUTOBUILD=1
OUT=gpurun_out/r3n
mkdir -p $OUT
timeout -k 10 120 python3 scripts/store_probe.py cuda 1000 breakdown > $OUT/breakdown_cuda.json 2> $OUT/err1.log &&
timeout -k 10 120 python3 scripts/store_probe.py cuda 1000 breakdown 150 > $OUT/breakdown_cuda_idle150.json 2> $OUT/err2.log &&
timeout -k 10 120 python3 scripts/store_probe.py host 1000 breakdown > $OUT/breakdown_host.json 2> $OUT/err3.log &&
echo done
