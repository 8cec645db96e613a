#!/bin/bash
# Render lanes grouped by record shape with co-located arena space (AHV_SP_ORDER=3) vs chain-only order (1).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp AHV_SKIP_AUTOBUILD=1
OUT=gpurun_out/r3v
mkdir -p $OUT
timeout -k 10 200 python -u -m pytest -x -q --timeout 150 --timeout-method thread -m gpu tests/test_store_pipeline.py tests/test_gpu_dist.py -k "hetero or pipeline" > $OUT/tests.log 2>&1 || { tail -20 $OUT/tests.log; exit 1; }
for o in 3 1 3 1; do
  AHV_SP_ORDER=$o timeout -k 10 200 python -u bench.py --mix hetero --sessions 1048576 --steps 10 --warmup 2 --no-scalar --no-api --no-liability > $OUT/ab_$o.json 2> $OUT/ab_$o.err || exit 1
  echo "$o $(python -c "import json;d=json.loads(open('$OUT/ab_$o.json').read().strip().splitlines()[-1]);print(d['value'],d['ms_per_step'])")" >> $OUT/ab.txt
done
AHV_SP_ORDER=3 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python -u bench.py --mix hetero --sessions 262144 --steps 5 --warmup 1 --no-scalar --no-api --no-liability > $OUT/prof.log 2>&1 || exit 1
echo done
