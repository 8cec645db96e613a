#!/bin/bash
# Round 4, call l: the wave-cooperative render kernel — batch tests (digests vs the
# scalar API, K10 re-verification), hetero bench A/B (coop vs lane renderer) at 1M
# and 4M sessions per step, a kernel trace and a lane-utilisation PMC pass.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp AHV_SKIP_AUTOBUILD=1
OUT=gpurun_out/r4l
mkdir -p $OUT
B="python bench.py --mix hetero --no-scalar --no-api --steps 20 --warmup 3"
timeout -k 10 400 python -u -m pytest tests/test_store_pipeline.py tests/test_batched_views.py tests/test_checkpoint.py -m gpu -x -q \
  -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 && echo tests-ok && \
timeout -k 10 300 $B --sessions 1048576 > $OUT/het1m_coop.log 2>&1 && echo h1c-ok && \
AHV_SP_RENDER=lane timeout -k 10 300 $B --sessions 1048576 > $OUT/het1m_lane.log 2>&1 && echo h1l-ok && \
timeout -k 10 300 $B > $OUT/het4m_coop.log 2>&1 && echo h4c-ok && \
AHV_SP_RENDER=lane timeout -k 10 300 $B > $OUT/het4m_lane.log 2>&1 && echo h4l-ok && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt -o kt -- python3 bench.py --mix hetero --no-scalar --no-api --steps 6 --warmup 2 --sessions 1048576 > $OUT/kt.log 2>&1 && echo kt-ok && \
timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_VALU SQ_THREAD_CYCLES_VALU SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_BUSY_CYCLES -d $OUT/pmc -o pmc -- python3 bench.py --mix hetero --no-scalar --no-api --steps 3 --warmup 1 --sessions 262144 > $OUT/pmc.log 2>&1 && echo pmc-ok && \
AHV_SP_RENDER=lane timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_VALU SQ_THREAD_CYCLES_VALU SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_BUSY_CYCLES -d $OUT/pmc_lane -o pmc -- python3 bench.py --mix hetero --no-scalar --no-api --steps 3 --warmup 1 --sessions 262144 > $OUT/pmc_lane.log 2>&1 && echo pmc-lane-ok
rc=$?
tail -2 $OUT/pytest.log
for f in het1m_coop het1m_lane het4m_coop het4m_lane; do echo $f; tail -1 $OUT/$f.log | cut -c1-260; done
exit $rc
