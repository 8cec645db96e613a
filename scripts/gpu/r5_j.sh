#!/bin/bash
# Round 5, call j: is the record tee slow because the payload arena is fine-grained?
# AB 2 tees into a coarse-grained scratch buffer instead (14: the same without SHA).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp AHV_SKIP_AUTOBUILD=1
OUT=gpurun_out/r5j
mkdir -p $OUT
B="python bench.py --steps 10 --warmup 2 --no-scalar --no-api --no-liability --verify-sessions 0"
for ab in 2 14; do
  AHV_TEMPLATE_AB=$ab timeout -k 10 300 $B > $OUT/ab$ab.log 2>&1 || exit $?
  echo "ab$ab $(tail -1 $OUT/ab$ab.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
