set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_store_lifecycle.py tests/test_gpu_store.py tests/test_store_fuzz.py > gpurun_out/g1_tests.log 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --scalar-iters 1000 > gpurun_out/g1_bench.log 2>&1
