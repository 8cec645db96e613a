#!/bin/bash
# Round 4, call ae: the 6.6 ms post_expect blocks in create_session — how far the
# worker lags behind the host before each pipeline (commands posted, not yet run),
# default worker vs no provisional Merkle roots vs no batched hashing.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp AHV_SKIP_AUTOBUILD=1
OUT=gpurun_out/r4ae
mkdir -p $OUT
timeout -k 10 300 python scripts/percall_outliers.py cuda 5000 > $OUT/outliers.txt 2>&1 && echo a-ok && \
AHV_STORE_SPECULATE=0 timeout -k 10 300 python scripts/percall_outliers.py cuda 5000 > $OUT/outliers_nospec.txt 2>&1 && echo b-ok && \
AHV_STORE_BATCH=0 timeout -k 10 300 python scripts/percall_outliers.py cuda 5000 > $OUT/outliers_nobatch.txt 2>&1 && echo c-ok
rc=$?
for f in outliers outliers_nospec outliers_nobatch; do echo "== $f"; sed -n 2,10p $OUT/$f.txt | cut -c1-200; done
exit $rc
