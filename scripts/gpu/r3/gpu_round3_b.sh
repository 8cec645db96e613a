set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/g2_tests.log 2>&1 && \
timeout -k 10 300 python -u benchmarks/bench_api.py --device cuda --n 10000 --rounds 3 --host > gpurun_out/g2_api.log 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --scalar-iters 1000 > gpurun_out/g2_bench.log 2>&1
