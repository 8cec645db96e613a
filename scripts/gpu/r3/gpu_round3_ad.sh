#!/bin/bash
# Headline step size: 1M vs 2M vs 4M sessions per GPU per step (same bench, liability stage included).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp AHV_SKIP_AUTOBUILD=1
OUT=gpurun_out/r3ad
mkdir -p $OUT
for s in 1048576 4194304 2097152 1048576 4194304; do
  timeout -k 10 200 python -u bench.py --sessions $s --no-scalar --no-api > $OUT/b_$s.json 2> $OUT/b_$s.err || exit 1
  echo "$s $(python -c "import json;d=json.loads(open('$OUT/b_$s.json').read().strip().splitlines()[-1]);print(d['value'],d['ms_per_step'],d['batch_p50_ms'])")" >> $OUT/ab.txt
done
echo done
