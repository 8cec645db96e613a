#!/bin/bash
# Round 6, call as: PMC of the batched heterogeneous kernels on the final layout (render+rows / prefix /
# chain with Merkle roots) at 1 M sessions per step — what bounds each.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp AHV_SKIP_AUTOBUILD=1
OUT=gpurun_out/r6as
mkdir -p $OUT
B="python bench.py --mix hetero --sessions 1048576 --steps 2 --warmup 1 --no-scalar --no-api --no-liability --verify-sessions 0"
P1="SQ_WAVES,SQ_WAVE_CYCLES,SQ_BUSY_CYCLES,SQ_INSTS_VALU,SQ_INSTS_SALU,SQ_INSTS_LDS,SQ_WAIT_INST_ANY,SQ_WAIT_ANY"
P2="SQ_INSTS_VMEM_WR,SQ_INSTS_VMEM_RD,SQ_INSTS_SMEM,SQ_ACTIVE_INST_VALU,SQ_ACTIVE_INST_LDS,SQ_WAIT_INST_LDS,SQ_INST_CYCLES_VMEM_WR,SQ_INST_CYCLES_VMEM_RD"
for p in 1 2; do
  if [ $p -eq 1 ]; then C=$P1; else C=$P2; fi
  timeout -s KILL 300 rocprofv3 --pmc $C -d $OUT/pmc_p$p -o run --output-format csv -- $B > $OUT/pmc_p$p.log 2>&1 || exit $?
  echo "pass $p ok"
done
find $OUT -name "*counter_collection.csv" | head
