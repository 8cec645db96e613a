#!/bin/bash
# Round 6, call z: small-value emit_uint fast path — batched pipeline GPU tests,
# hetero bench (1 M / 4 M per step), headline without the API section, and the
# BASELINE configs 2-5 on the final build; command-wave slot prefetch A/B.
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
# command-wave slot prefetch A/B: default (issued before execution), off, late (after publication)
for mode in default off late; do
  case $mode in default) E="";; off) E="AHV_STORE_SLOT_PREFETCH=0";; late) E="AHV_STORE_LATE_PREFETCH=1";; esac
  env $E timeout -k 10 200 python scripts/probe_worker.py > $OUT/probe_$mode.json 2>$OUT/probe_$mode.err || exit $?
  env $E ITERS=2000 timeout -k 10 200 python scripts/profile_percall.py > $OUT/percall_$mode.txt 2>&1 || exit $?
  echo "$mode $(tail -1 $OUT/probe_$mode.json | cut -c1-150) p50 $(head -2 $OUT/percall_$mode.txt | tail -1 | cut -c40-75)"
done
