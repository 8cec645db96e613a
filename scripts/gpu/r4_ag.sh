#!/bin/bash
# Round 4, call ag: worker feature bits keep results (tests/test_worker_features.py) and the lifecycle tests.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp AHV_SKIP_AUTOBUILD=1
OUT=gpurun_out/r4ag
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_worker_features.py tests/test_store_lifecycle.py -m gpu -x -v \
  -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 && echo tests-ok
rc=$?
grep -E "PASS|FAIL|ERROR|passed|failed" $OUT/pytest.log | tail -12
exit $rc
