set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 1100 python -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu tests/ > gpurun_out/g4_tests.log 2>&1
rc=$?; echo "tests rc=$rc" >> gpurun_out/g4_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u benchmarks/bench_api.py --device cuda --n 10000 --rounds 3 --host --batch 100000 > gpurun_out/g4_api.log 2>&1
