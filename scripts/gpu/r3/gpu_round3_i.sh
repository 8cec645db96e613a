#!/bin/bash
# Register-form render, device touched list, slash_clip rewrite: tests, config5, headline bench, trace.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp AHV_SKIP_AUTOBUILD=1
OUT=gpurun_out/r3i
mkdir -p $OUT
echo "[r3i] $(date +%T) tests"
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_kernels.py tests/test_config5_arena.py tests/test_global_liability.py > $OUT/tests.log 2>&1 || { echo "tests failed"; tail -30 $OUT/tests.log; exit 1; }
echo "[r3i] $(date +%T) config5"
for v in 1 2 3; do
  timeout -k 10 200 python -u benchmarks/bench_configs.py config5 --steps 10 --warmup 2 > $OUT/c5_$v.log 2>&1 || exit 1
  echo "run $v $(grep -o '"ms_per_storm": [0-9.]*' $OUT/c5_$v.log)" >> $OUT/c5_summary.txt
done
echo "[r3i] $(date +%T) bench"
timeout -k 10 300 python -u bench.py --no-api > $OUT/bench1.log 2>&1 &&
timeout -k 10 300 python -u bench.py --no-api --no-liability --no-scalar > $OUT/bench_noliab.log 2>&1 &&
timeout -k 10 300 python -u bench.py --no-api --no-scalar > $OUT/bench2.log 2>&1 || exit 1
echo "[r3i] $(date +%T) traces"
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_c5 -o c5 -- python3 benchmarks/bench_configs.py config5 --steps 10 --warmup 2 > $OUT/trace_c5.log 2>&1 || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_bench -o b -- python3 bench.py --steps 10 --warmup 2 --no-scalar --no-api > $OUT/trace_bench.log 2>&1 || exit 1
echo "[r3i] $(date +%T) done"
