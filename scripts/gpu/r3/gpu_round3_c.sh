set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 1000 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/g3_tests.log 2>&1
rc=$?
echo "tests rc=$rc" >> gpurun_out/g3_tests.log
[ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_api -o api -- python3 benchmarks/bench_api.py --device cuda --n 4000 --rounds 1 > gpurun_out/g3_api_prof.log 2>&1
