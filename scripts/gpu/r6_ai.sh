#!/bin/bash
# Round 6, call ai: final build after the batch-kernel changes (render-first layout,
# chain-lane Merkle roots, straight-line arena sink) — full GPU suite, default bench,
# hetero at 1 M / 4 M per step, configs 2-5.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp AHV_SKIP_AUTOBUILD=1
OUT=gpurun_out/r6ai
mkdir -p $OUT
timeout -k 10 800 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/gpu_tests.txt 2>&1; rc=$?
tail -2 $OUT/gpu_tests.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py > $OUT/bench.json 2> $OUT/bench.err || exit $?
tail -1 $OUT/bench.json | cut -c1-300
for S in 1048576 4194304; do
  timeout -k 10 300 python bench.py --mix hetero --no-scalar --no-api --sessions $S --steps 20 --warmup 3 > $OUT/hetero_$S.json 2>$OUT/hetero_$S.err || exit $?
  echo "hetero S=$S $(tail -1 $OUT/hetero_$S.json | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
timeout -k 10 600 python benchmarks/bench_configs.py config2 config3 config4 config5 > $OUT/configs.jsonl 2> $OUT/configs.err || exit $?
cut -c1-200 $OUT/configs.jsonl
