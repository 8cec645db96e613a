#!/bin/bash
# Heterogeneous-mix bench (bench.py --mix hetero) + its kernel trace; default bench for p50 after the
# per-call micro-optimisations.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp AHV_SKIP_AUTOBUILD=1
OUT=gpurun_out/r3o
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_dist.py tests/test_store_pipeline.py > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
timeout -k 10 300 python -u bench.py --mix hetero --sessions 1048576 --steps 10 --warmup 2 --no-scalar --no-api > $OUT/hetero_1m.json 2> $OUT/hetero_1m.err || exit 1
timeout -k 10 300 python -u bench.py --mix hetero --sessions 262144 --steps 10 --warmup 2 --no-scalar --no-api --no-liability > $OUT/hetero_256k_noliab.json 2> $OUT/hetero_256k.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_hetero -o run -- python -u bench.py --mix hetero --sessions 262144 --steps 5 --warmup 1 --no-scalar --no-api > $OUT/prof_hetero.log 2>&1 || exit 1
timeout -k 10 400 python -u bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err || exit 1
echo done
