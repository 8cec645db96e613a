#!/bin/bash
# Round 4, call c: A/B of the template kernel's record tee (none / fine-grained arena /
# coarse scratch) and of the participant row width.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp AHV_SKIP_AUTOBUILD=1
OUT=gpurun_out/r4c
mkdir -p $OUT
B="python bench.py --steps 10 --warmup 2 --no-scalar --no-api --no-liability"
for cfg in "0 16" "1 16" "2 16" "0 10" "0 4"; do
  set -- $cfg
  AHV_TEMPLATE_AB=$1 timeout -k 10 300 $B --participant-rows $2 > $OUT/ab_$1_p$2.log 2>&1 || exit $?
  echo "ab=$1 P=$2 $(python -c "import json,sys; d=json.loads(open('$OUT/ab_$1_p$2.log').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'])")"
done
