#!/bin/bash
# Round 6, call at: what the liability stage (K04 exposure + K06 slash + X02, side stream)
# costs the timed step — headline template and hetero at 1 M, with and without it
# (--no-liability), plus kernel stats of the liability kernels alone.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp AHV_SKIP_AUTOBUILD=1
OUT=gpurun_out/r6at
mkdir -p $OUT
for rep in 1 2; do
  for L in "" "--no-liability"; do
    tag=${L:+noliab}; tag=${tag:-liab}
    timeout -k 10 300 python bench.py --no-scalar --no-api $L > $OUT/t_${tag}_$rep.json 2>$OUT/t_${tag}_$rep.err || exit $?
    timeout -k 10 300 python bench.py --mix hetero --no-scalar --no-api --sessions 1048576 --steps 20 --warmup 3 $L > $OUT/h_${tag}_$rep.json 2>$OUT/h_${tag}_$rep.err || exit $?
    echo "rep=$rep $tag template $(tail -1 $OUT/t_${tag}_$rep.json | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])') hetero $(tail -1 $OUT/h_${tag}_$rep.json | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
