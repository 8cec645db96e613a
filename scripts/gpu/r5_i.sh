#!/bin/bash
# Round 5, call i: headline kernel variants with the changes fragments — tee cost (AB 1),
# tee + SHA (AB 13), one-pass window <1,6> at 4M, <2,3>, <4,2>.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp AHV_SKIP_AUTOBUILD=1
OUT=gpurun_out/r5i
mkdir -p $OUT
B="python bench.py --steps 10 --warmup 2 --no-scalar --no-api --no-liability --verify-sessions 0"
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 300 $B > $OUT/$name.log 2>&1 || return $?
  echo "$name $(tail -1 $OUT/$name.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
}
run ab1 AHV_TEMPLATE_AB=1 && run ab13 AHV_TEMPLATE_AB=13 && run w16 AHV_TEMPLATE_SMALL=16777216 && \
run w2 AHV_TEMPLATE_WAVES=2 && run w4 AHV_TEMPLATE_WAVES=4 && run base AHV_TEMPLATE_AB=0
timeout -k 10 300 python benchmarks/bench_api.py --device cuda --n 200 --batch 20000 --rounds 5 > $OUT/api.json 2>&1 || exit $?
tail -1 $OUT/api.json | python -c 'import json,sys; d=json.loads(sys.stdin.read()); [print(k, d[k].get("sessions_per_s"), d[k].get("phases_ms")) for k in ("batch","batch_hetero")]'
