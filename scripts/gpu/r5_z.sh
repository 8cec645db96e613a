#!/bin/bash
# Round 5, call z: hetero batch end to end by spec-walk thread count.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp AHV_SKIP_AUTOBUILD=1
OUT=gpurun_out/r5z
mkdir -p $OUT
for th in 16 8 4 16 8 4; do
  AHV_PACK_THREADS=$th timeout -k 10 300 python benchmarks/bench_api.py --n 0 --batch 20000 --rounds 7 > $OUT/api_t$th.json 2>&1 || exit $?
  echo "t$th $(grep -v amdgpu $OUT/api_t$th.json | tail -1 | python -c 'import json,sys; d=json.loads(sys.stdin.read())["batch_hetero"]; print(d["sessions_per_s"], d["phases_ms"])')"
done
