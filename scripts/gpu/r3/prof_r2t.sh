#!/bin/bash
# config5 A/B: K08 midstate split and the fused slash + sigma_eff pass (kernel
# tests, storm time, kernel traces).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp AHV_SKIP_AUTOBUILD=1
OUT=gpurun_out/r2t
mkdir -p $OUT
C5="python3 benchmarks/bench_configs.py config5 --steps 10 --warmup 2"
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 &&
timeout -k 10 200 $C5 > $OUT/c5_new.log 2>&1 &&
timeout -k 10 200 $C5 --no-midstate > $OUT/c5_nomid.log 2>&1 &&
timeout -k 10 200 $C5 --unfused > $OUT/c5_unfused.log 2>&1 &&
timeout -k 10 200 $C5 --unfused --no-midstate > $OUT/c5_old.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_new -o run -- $C5 > $OUT/trace_new.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_old -o run -- $C5 --unfused --no-midstate > $OUT/trace_old.log 2>&1
