#!/bin/bash
# Round 4, call q: the rows kernel without read-after-write round trips — batch tests
# (incl. every layout switch), hetero bench at 1M and 4M, a kernel trace at 1M.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp AHV_SKIP_AUTOBUILD=1
OUT=gpurun_out/r4q
mkdir -p $OUT
B="python bench.py --mix hetero --no-scalar --no-api --steps 20 --warmup 3"
timeout -k 10 900 python -u -m pytest tests/test_store_pipeline.py tests/test_batched_views.py -m gpu -x -q \
  -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 && echo tests-ok && \
timeout -k 10 300 $B --sessions 1048576 > $OUT/h1m.log 2>&1 && echo h1m-ok && \
timeout -k 10 300 $B > $OUT/h4m.log 2>&1 && echo h4m-ok && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt -o kt -- python3 bench.py --mix hetero --no-scalar --no-api --steps 6 --warmup 2 --sessions 1048576 > $OUT/kt.log 2>&1 && echo kt-ok && \
python scripts/prof_summary.py $(find $OUT/kt -name "*.db" | head -1) > $OUT/kt.md && \
timeout -k 10 200 python scripts/percall_split.py cuda > $OUT/split_cuda.txt 2>&1 && echo split-ok && \
timeout -k 10 200 python scripts/percall_split.py host > $OUT/split_host.txt 2>&1 && echo split-host-ok
rc=$?
rm -rf $OUT/kt
tail -1 $OUT/pytest.log
for f in h1m h4m; do echo $f; tail -1 $OUT/$f.log | cut -c1-200; done
head -12 $OUT/kt.md | cut -c1-160
cat $OUT/split_cuda.txt $OUT/split_host.txt
exit $rc
