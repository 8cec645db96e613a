#!/bin/bash
# Round 6, call x: public batched API (template and heterogeneous, 2·10^4 and 10^5
# sessions) with the record-head fragments on and off (AHV_SP_FRAGS).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp AHV_SKIP_AUTOBUILD=1
OUT=gpurun_out/r6x
mkdir -p $OUT
for fr in 0 1; do
  AHV_SP_FRAGS=$fr timeout -k 10 300 python -c "
import json, sys
sys.path.insert(0, '.')
from benchmarks.bench_api import batch_api_throughput
for n in (20000, 100000):
    r = batch_api_throughput('cuda', n, 3, hetero=True)
    r.pop('rounds', None)
    print(json.dumps(dict(r, frags=$fr)))
" > $OUT/hetero_api_f$fr.jsonl 2> $OUT/hetero_api_f$fr.err || exit $?
  cat $OUT/hetero_api_f$fr.jsonl | cut -c1-300
done
