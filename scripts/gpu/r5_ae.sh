#!/bin/bash
# Round 5, call ae: RCCL at world 2 with both ranks on the box's one GPU.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp AHV_SKIP_AUTOBUILD=1
OUT=gpurun_out/r5ae
mkdir -p $OUT
timeout -k 10 180 python -m torch.distributed.run --nnodes 1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29533 scripts/rccl_two_ranks_one_gpu.py > $OUT/rccl2.log 2>&1; rc=$?
grep -v amdgpu $OUT/rccl2.log | grep -E '^\{|rror|refused' | head -10 | cut -c1-600
exit $rc
