#!/bin/bash
# Headline A/B: liability side stream joined every step (old) vs unjoined (new).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp AHV_SKIP_AUTOBUILD=1
OUT=gpurun_out/r2y
mkdir -p $OUT
for i in 1 2; do
  timeout -k 10 120 python3 bench.py --no-scalar > $OUT/new_$i.log 2>&1 &&
  timeout -k 10 120 python3 bench.py --no-scalar --join-liability > $OUT/old_$i.log 2>&1 || exit $?
done
timeout -k 10 300 python3 bench.py > $OUT/bench.log 2>&1 &&
timeout -k 10 200 python3 -u -m pytest tests/test_gpu_dist.py -x -q --timeout 120 --timeout-method thread > $OUT/dist.log 2>&1 &&
timeout -k 10 300 python3 scripts/saga_runner_prof.py cuda > $OUT/saga_prof.log 2>&1
