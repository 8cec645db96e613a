#!/bin/bash
# Capacity sweep: resident liability graphs of 1M-64M agents, pipeline launches of 1M-8M sessions.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp AHV_SKIP_AUTOBUILD=1
OUT=gpurun_out/r3ac
mkdir -p $OUT
timeout -k 10 400 python -u benchmarks/bench_capacity.py > $OUT/capacity.jsonl 2> $OUT/capacity.err || { tail -5 $OUT/capacity.err; exit 1; }
echo done
