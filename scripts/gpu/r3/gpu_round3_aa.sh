#!/bin/bash
# Kernel traces of BASELINE configs 2 and 3 (what bounds a 10k-session step).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp AHV_SKIP_AUTOBUILD=1
OUT=gpurun_out/r3aa
mkdir -p $OUT
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/c2 -o run -- python -u benchmarks/bench_configs.py config2 > $OUT/c2.log 2>&1 || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/c3 -o run -- python -u benchmarks/bench_configs.py config3 > $OUT/c3.log 2>&1 || exit 1
echo done
