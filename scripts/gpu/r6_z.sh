#!/bin/bash
# Round 6, call z: small-value emit_uint fast path — batched pipeline GPU tests,
# hetero bench (1 M / 4 M per step), headline without the API section, and the
# BASELINE configs 2-5 on the final build.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp AHV_SKIP_AUTOBUILD=1
OUT=gpurun_out/r6z
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_store_pipeline.py tests/test_gpu_pipeline.py tests/test_gpu_headline_oracle.py tests/test_store_template.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/tests.txt 2>&1; rc=$?
tail -2 $OUT/tests.txt; [ $rc -eq 0 ] || exit $rc
for S in 1048576 4194304; do
  timeout -k 10 300 python bench.py --mix hetero --no-scalar --no-api --sessions $S --steps 10 --warmup 2 > $OUT/hetero_$S.json 2>$OUT/hetero_$S.err || exit $?
  echo "hetero S=$S $(tail -1 $OUT/hetero_$S.json | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
timeout -k 10 300 python bench.py --no-scalar --no-api > $OUT/headline.json 2>$OUT/headline.err || exit $?
echo "headline $(tail -1 $OUT/headline.json | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["headline_verified"])')"
timeout -k 10 600 python benchmarks/bench_configs.py config2 config3 config4 config5 > $OUT/configs.jsonl 2> $OUT/configs.err || exit $?
cut -c1-220 $OUT/configs.jsonl
