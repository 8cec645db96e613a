#!/bin/bash
# Where the parent-independent SHA blocks go: render lane (default) vs the work-sorted chain lane (no split).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp AHV_SKIP_AUTOBUILD=1
OUT=gpurun_out/r3w
mkdir -p $OUT
for m in render chain render chain; do
  AHV_SP_PREFIX=$m timeout -k 10 200 python -u bench.py --mix hetero --sessions 1048576 --steps 10 --warmup 2 --no-scalar --no-api --no-liability > $OUT/ab_$m.json 2> $OUT/ab_$m.err || exit 1
  echo "$m $(python -c "import json;d=json.loads(open('$OUT/ab_$m.json').read().strip().splitlines()[-1]);print(d['value'],d['ms_per_step'])")" >> $OUT/ab.txt
done
echo done
