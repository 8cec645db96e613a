#!/bin/bash
# Round 5, call ag: root stress with the final worker and API (awaited terminate with
# overlapped bookkeeping), 2 × 6,000 sessions of 1-8 captures.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp AHV_SKIP_AUTOBUILD=1
OUT=gpurun_out/r5ag
mkdir -p $OUT
for k in 1 2; do
  timeout -k 10 200 python scripts/root_stress.py 6000 cuda > $OUT/stress$k.txt 2>&1 || exit $?
  tail -1 $OUT/stress$k.txt | cut -c1-300
done
