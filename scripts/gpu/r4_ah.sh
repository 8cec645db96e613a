#!/bin/bash
# Round 4, call ah: the hetero chain kernel writes each parent digest's hex as 16-17
# aligned word stores instead of 64 byte stores — batch tests, hetero bench at 1M and
# 4M, a kernel trace at 1M (chain kernel was 431 us at 1M in r4q).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp AHV_SKIP_AUTOBUILD=1
OUT=gpurun_out/r4ah
mkdir -p $OUT
B="python bench.py --mix hetero --no-scalar --no-api --steps 20 --warmup 3"
timeout -k 10 900 python -u -m pytest tests/test_store_pipeline.py tests/test_batched_views.py -m gpu -x -q \
  -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 && echo tests-ok && \
timeout -k 10 300 $B --sessions 1048576 > $OUT/h1m.log 2>&1 && echo h1m-ok && \
timeout -k 10 300 $B > $OUT/h4m.log 2>&1 && echo h4m-ok && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt -o kt -- python3 bench.py --mix hetero --no-scalar --no-api --steps 6 --warmup 2 --sessions 1048576 > $OUT/kt.log 2>&1 && echo kt-ok && \
python scripts/prof_summary.py $(find $OUT/kt -name "*.db" | head -1) > $OUT/kt.md
rc=$?
rm -rf $OUT/kt
tail -1 $OUT/pytest.log
for f in h1m h4m; do echo $f; tail -1 $OUT/$f.log | cut -c1-200; done
head -10 $OUT/kt.md | cut -c1-160
exit $rc
