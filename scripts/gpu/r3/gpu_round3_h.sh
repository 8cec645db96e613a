#!/bin/bash
# Round-3 checkpoint: all GPU tests, engines at 100k calls, config4/5 (slash modes), bench.py with the
# API section, kernel traces of config5 and of the batched API, slash counters.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp AHV_SKIP_AUTOBUILD=1
OUT=gpurun_out/r3h
mkdir -p $OUT
echo "[r3h] $(date +%T) tests"
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ > $OUT/tests.log 2>&1 || { echo "tests failed"; tail -30 $OUT/tests.log; exit 1; }
echo "[r3h] $(date +%T) engines"
timeout -k 10 300 python -u benchmarks/bench_engines.py > $OUT/engines.log 2>&1 || exit 1
echo "[r3h] $(date +%T) config4/5"
timeout -k 10 300 python -u benchmarks/bench_configs.py config4 --steps 5 --warmup 2 > $OUT/c4.log 2>&1 || exit 1
for v in 0 3 0; do
  AHV_SLASH_MODE=$v timeout -k 10 200 python -u benchmarks/bench_configs.py config5 --steps 10 --warmup 2 > $OUT/c5_m$v.log 2>&1 || exit 1
  echo "mode $v $(grep -o '"ms_per_storm": [0-9.]*' $OUT/c5_m$v.log)" >> $OUT/c5_summary.txt
done
echo "[r3h] $(date +%T) bench"
timeout -k 10 600 python -u bench.py > $OUT/bench.log 2>&1 || exit 1
echo "[r3h] $(date +%T) traces"
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_c5 -o c5 -- python3 benchmarks/bench_configs.py config5 --steps 10 --warmup 2 > $OUT/trace_c5.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_api -o api -- python3 benchmarks/bench_api.py --device cuda --n 0 --batch 100000 --rounds 3 > $OUT/trace_api.log 2>&1 || exit 1
echo "[r3h] $(date +%T) pmc"
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM SQ_INSTS_LDS SQ_INSTS_SALU --kernel-include-regex "slash|sigma|exposure" --output-format csv -d $OUT/pmc_stall -o pmc -- python3 benchmarks/bench_liability.py --iters 3 --sessions 1250000 --only exposure,stream,csr,slash_split > $OUT/pmc_stall.log 2>&1
echo "[r3h] $(date +%T) done"
