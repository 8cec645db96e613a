#!/bin/bash
# Round 6, call bg: final round-end rehearsal on the final tree (spill-free render+rows kernel) — smoke(), the full GPU suite,
# the default 1-GPU bench and `bench.py --gpus 1` as the driver launches it.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp AHV_SKIP_AUTOBUILD=1
OUT=gpurun_out/r6bg
mkdir -p $OUT
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.txt 2>&1 || { tail -5 $OUT/smoke.txt; exit 1; }
tail -1 $OUT/smoke.txt
timeout -k 10 800 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/gpu_tests.txt 2>&1; rc=$?
tail -2 $OUT/gpu_tests.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py > $OUT/bench.json 2> $OUT/bench.err || exit $?
tail -1 $OUT/bench.json | cut -c1-250
timeout -k 10 400 python bench.py --gpus 1 --steps 10 --warmup 2 > $OUT/bench_g1.json 2> $OUT/bench_g1.err || exit $?
tail -1 $OUT/bench_g1.json | cut -c1-250
for S in 1048576 4194304; do
  timeout -k 10 300 python bench.py --mix hetero --no-scalar --no-api --sessions $S --steps 20 --warmup 3 > $OUT/hetero_$S.json 2>$OUT/hetero_$S.err || exit $?
  echo "hetero S=$S $(tail -1 $OUT/hetero_$S.json | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
timeout -k 10 600 python benchmarks/bench_configs.py config2 config3 config4 config5 > $OUT/configs.jsonl 2> $OUT/configs.err || exit $?
cut -c1-160 $OUT/configs.jsonl
