#!/bin/bash
# The driver's default bench invocation (python bench.py) after the step-size change, and the gloo-free
# one-rank RCCL path (AHV_BENCH_FORCE_DIST) at the new default.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp AHV_SKIP_AUTOBUILD=1
OUT=gpurun_out/r3ae
mkdir -p $OUT
timeout -k 10 600 python -u bench.py > $OUT/bench.log 2>&1 || { tail -20 $OUT/bench.log; exit 1; }
AHV_BENCH_FORCE_DIST=1 timeout -k 10 300 python -u -m torch.distributed.run --standalone --local-addr 127.0.0.1 --nnodes=1 --nproc-per-node 1 bench.py --no-scalar --no-api > $OUT/bench_dist1.log 2>&1 || { tail -20 $OUT/bench_dist1.log; exit 1; }
echo done
