#!/bin/bash
# config5 kernel counters (one pass per counter group): instruction mix / stalls,
# HBM fetch, HBM write — for the fused slash/σ_eff, K08 prefix + serial pass,
# render_rows and Merkle kernels.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp AHV_SKIP_AUTOBUILD=1
OUT=gpurun_out/r3b
mkdir -p $OUT
C5="python3 benchmarks/bench_configs.py config5 --steps 2 --warmup 1"
RX="slash|chain|render|merkle"
pmc() {
  local name=$1 ctr=$2
  echo "[prof_r3b] $(date +%T) pmc $name"
  timeout -s KILL 150 rocprofv3 --pmc $ctr --kernel-include-regex "$RX" --output-format csv -d $OUT/pmc_$name -o pmc -- $C5 > $OUT/pmc_$name.log 2>&1
}
pmc stall "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM SQ_INSTS_LDS SQ_INSTS_SALU" &&
pmc fetch "FETCH_SIZE GRBM_GUI_ACTIVE" &&
pmc write "WRITE_SIZE GRBM_GUI_ACTIVE"
