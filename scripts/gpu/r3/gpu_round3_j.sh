#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp AHV_SKIP_AUTOBUILD=1
OUT=gpurun_out/r3j
mkdir -p $OUT
echo "[r3j] $(date +%T) tests"
timeout -k 10 600 python -u -m pytest -x -q --timeout 400 --timeout-method thread -m gpu tests/test_config5_arena.py tests/test_store_pipeline.py tests/test_gpu_kernels.py > $OUT/tests.log 2>&1 || { echo "tests failed"; tail -30 $OUT/tests.log; exit 1; }
echo "[r3j] $(date +%T) config5"
for v in 1 2 3; do
  timeout -k 10 200 python -u benchmarks/bench_configs.py config5 --steps 10 --warmup 2 > $OUT/c5_$v.log 2>&1 || exit 1
  echo "run $v $(grep -o '"ms_per_storm": [0-9.]*' $OUT/c5_$v.log)" >> $OUT/c5_summary.txt
done
echo "[r3j] $(date +%T) config2_api"
timeout -k 10 400 python -u benchmarks/bench_configs.py config2_api --steps 6 > $OUT/c2api.log 2>&1 || exit 1
echo "[r3j] $(date +%T) trace"
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_c5 -o c5 -- python3 benchmarks/bench_configs.py config5 --steps 10 --warmup 2 > $OUT/trace_c5.log 2>&1 || exit 1
echo "[r3j] $(date +%T) done"
