#!/bin/bash
# Round 5, call g: PMC passes on the headline kernel (full vs no-SHA A/B) and the
# per-call awaited timeline with a longer busy-loop spin for results.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp AHV_SKIP_AUTOBUILD=1
OUT=gpurun_out/r5g
mkdir -p $OUT
B="python bench.py --steps 2 --warmup 1 --no-scalar --no-api --no-liability --verify-sessions 0"
P1="SQ_WAVES,SQ_WAVE_CYCLES,SQ_BUSY_CYCLES,SQ_INSTS_VALU,SQ_INSTS_SALU,SQ_INSTS_LDS,SQ_WAIT_INST_ANY,SQ_WAIT_ANY"
P2="SQ_INSTS_VMEM_WR,SQ_INSTS_VMEM_RD,SQ_INSTS_SMEM,SQ_ACTIVE_INST_VALU,SQ_ACTIVE_INST_LDS,SQ_WAIT_INST_LDS,SQ_INST_CYCLES_VMEM_WR,SQ_INST_CYCLES_VMEM_RD"
for ab in 0 12; do
  for p in 1 2; do
    if [ $p -eq 1 ]; then C=$P1; else C=$P2; fi
    AHV_TEMPLATE_AB=$ab timeout -s KILL 300 rocprofv3 --pmc $C -d $OUT/pmc_ab${ab}_p$p -o run --output-format csv -- $B \
      > $OUT/pmc_ab${ab}_p$p.log 2>&1 || exit $?
    echo "ab=$ab pass=$p ok"
  done
done
AHV_SPEC_TERMINATE=0 AHV_STORE_SPIN_BUSY_NS=150000 timeout -k 10 300 python scripts/percall_timeline.py > $OUT/timeline_awaited_spin.jsonl 2>&1
rc=$?
grep -v amdgpu $OUT/timeline_awaited_spin.jsonl | head -3
find $OUT -name "*counter_collection.csv" | head
exit $rc
