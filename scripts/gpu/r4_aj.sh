#!/bin/bash
# Round 4, call aj: headline kernel occupancy A/B — <3,3> (default, 3 waves/SIMD, LDS-bound)
# vs <4,2> (2-block window, 4 waves/SIMD, one more emission pass); headline bench at 4 M.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp AHV_SKIP_AUTOBUILD=1
OUT=gpurun_out/r4aj
mkdir -p $OUT
B="python bench.py --steps 20 --warmup 3 --no-scalar --no-api"
timeout -k 10 300 python -u -m pytest tests/test_gpu_resources.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 && echo res-ok && \
timeout -k 10 300 $B > $OUT/w3.log 2>&1 && echo w3-ok && \
AHV_TEMPLATE_WAVES=4 timeout -k 10 300 $B > $OUT/w4.log 2>&1 && echo w4-ok && \
timeout -k 10 300 $B > $OUT/w3b.log 2>&1 && echo w3b-ok && \
AHV_TEMPLATE_WAVES=4 timeout -k 10 300 $B > $OUT/w4b.log 2>&1 && echo w4b-ok
rc=$?
tail -1 $OUT/pytest.log
for f in w3 w4 w3b w4b; do echo $f; tail -1 $OUT/$f.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['last_step_counters'])"; done
exit $rc
