#!/bin/bash
# A/B of the batch kernels' work layout (lane orders, prefix SHA placement) on the hetero mix.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp AHV_SKIP_AUTOBUILD=1
OUT=gpurun_out/r3r
mkdir -p $OUT
for v in "1 render" "3 render" "1 kernel" "0 render" "1 render"; do
  set -- $v
  AHV_SP_ORDER=$1 AHV_SP_PREFIX=$2 timeout -k 10 200 python -u bench.py --mix hetero --sessions 1048576 --steps 10 --warmup 2 --no-scalar --no-api --no-liability > $OUT/ab_$1_$2.json 2> $OUT/ab_$1_$2.err || exit 1
  echo "$1 $2 $(python -c "import json;d=json.loads(open('$OUT/ab_$1_$2.json').read().strip().splitlines()[-1]);print(d['value'],d['ms_per_step'])")" >> $OUT/ab.txt
done
echo done
