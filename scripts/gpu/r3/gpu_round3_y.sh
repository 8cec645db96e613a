#!/bin/bash
# Per-call gather: spin-before-suspend when other tasks are ready (AHV_STORE_SPIN_BUSY_NS) A/B.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp AHV_SKIP_AUTOBUILD=1
OUT=gpurun_out/r3y2
mkdir -p $OUT
for ns in 10000 20000 40000 80000 20000 40000; do
  AHV_STORE_SPIN_BUSY_NS=$ns timeout -k 10 200 python -u -c "
import sys, json; sys.path.insert(0, '.'); sys.path.insert(0, 'benchmarks')
from bench_api import api_throughput
print(json.dumps(dict(spin_busy_ns=$ns, **api_throughput('cuda', 10000, rounds=3))))" >> $OUT/spin.jsonl 2> $OUT/err.log || exit 1
done
echo done
