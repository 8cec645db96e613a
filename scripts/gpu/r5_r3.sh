#!/bin/bash
# Round 5, call r3: round-end rehearsal (after the close reorder) — the whole GPU suite, smoke(), then the default bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp AHV_SKIP_AUTOBUILD=1
OUT=gpurun_out/r5r3
mkdir -p $OUT
timeout -k 10 1200 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread \
  > $OUT/gpu_tests.log 2>&1; rc=$?
tail -5 $OUT/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 || exit $?
tail -1 $OUT/smoke.log
timeout -k 10 600 python bench.py > $OUT/bench.json 2>$OUT/bench.err; rc=$?
tail -1 $OUT/bench.json | cut -c1-3000
exit $rc
