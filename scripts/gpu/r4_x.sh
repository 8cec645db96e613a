#!/bin/bash
# Round 4, call x: how often the host finds the command ring full (worker behind) in
# back-to-back per-call pipelines and under asyncio.gather.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp AHV_SKIP_AUTOBUILD=1
OUT=gpurun_out/r4x
mkdir -p $OUT
ITERS=3000 timeout -k 10 300 python scripts/profile_percall.py > $OUT/percall.log 2>&1 && echo percall-ok && \
N=10000 timeout -k 10 300 python scripts/profile_gather.py > $OUT/gather.log 2>&1 && echo gather-ok
rc=$?
grep p50_us $OUT/percall.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); i=d['store_info_delta']; print({k: d[k] for k in ('p50_us','mean_us','host_cpu_us_per_pipeline')}, 'ring_waits', i.get('ring_waits'), 'ring_wait_us/pipeline', i.get('ring_wait_us',0)/d['iters'])"
head -3 $OUT/gather.log | cut -c1-250
exit $rc
