#!/bin/bash
# Round 4, call g: worker probes (per-call critical path), the headline with
# participant-major columns, MFMA PMC on the config3 sigma/exposure path.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp AHV_SKIP_AUTOBUILD=1
OUT=gpurun_out/r4g
mkdir -p $OUT
timeout -k 10 300 python scripts/probe_worker.py > $OUT/probe.log 2>&1 && echo probe-ok && \
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-scalar --no-api > $OUT/bench_a.log 2>&1 && echo bench-a-ok && \
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-scalar --no-api > $OUT/bench_b.log 2>&1 && echo bench-b-ok && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run -- python bench.py --steps 10 --warmup 2 --no-scalar --no-api > $OUT/prof.log 2>&1 && echo prof-ok && \
timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_INSTS_VALU -d $OUT/pmc -o mfma -- python benchmarks/bench_mfma_ab.py --iters 20 > $OUT/pmc.log 2>&1 && echo pmc-ok
rc=$?
cat $OUT/probe.log | tail -1; tail -1 $OUT/bench_a.log | cut -c1-260; tail -1 $OUT/bench_b.log | cut -c1-260; tail -3 $OUT/pmc.log
exit $rc
