#!/bin/bash
# Round 6, call ar: BASELINE config 5 with the K07 bond release on a side stream beside the
# re-chain's SHA passes vs in line (--serial-release) — interleaved A/B, then config 5 and
# its 10 % subset as the default runs them.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp AHV_SKIP_AUTOBUILD=1
OUT=gpurun_out/r6ar
mkdir -p $OUT
for rep in 1 2 3; do
  for mode in side serial; do
    F=""; [ $mode = serial ] && F="--serial-release"
    timeout -k 10 300 python benchmarks/bench_configs.py config5 $F > $OUT/c5_${mode}_$rep.jsonl 2> $OUT/c5_${mode}_$rep.err || exit $?
    echo "rep=$rep release=$mode $(python -c 'import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d["ms_per_storm"], d["bond_updates"], d["release_stream"])' $OUT/c5_${mode}_$rep.jsonl)"
  done
done
