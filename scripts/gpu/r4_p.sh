#!/bin/bash
# Round 4, call p: config2 as one captured graph with the fused epilogue (A/B vs the
# unfused nodes), graph tests, hetero render-order A/B at 1M and the 4M hetero line.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp AHV_SKIP_AUTOBUILD=1
OUT=gpurun_out/r4p
mkdir -p $OUT
B="python bench.py --mix hetero --no-scalar --no-api --steps 20 --warmup 3"
timeout -k 10 300 python -u -m pytest tests/test_graphs.py tests/test_gpu_pipeline.py tests/test_gpu_resources.py tests/test_store_template.py -m gpu -x -q \
  -p no:cacheprovider --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1 && echo tests-ok && \
timeout -k 10 300 python benchmarks/bench_configs.py config2 --steps 50 --warmup 5 > $OUT/c2_fused.log 2>&1 && echo c2f-ok && \
timeout -k 10 300 python benchmarks/bench_configs.py config2 --steps 50 --warmup 5 --unfused-graph > $OUT/c2_unfused.log 2>&1 && echo c2u-ok && \
AHV_TEMPLATE_SMALL=0 timeout -k 10 300 python benchmarks/bench_configs.py config2 --steps 50 --warmup 5 > $OUT/c2_w3.log 2>&1 && echo c2w3-ok && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt -o kt -- python3 benchmarks/bench_configs.py config2 --steps 20 --warmup 3 > $OUT/kt.log 2>&1 && echo kt-ok && \
python scripts/prof_summary.py $(find $OUT/kt -name "*.db" | head -1) > $OUT/c2_kernels.md && \
AHV_SP_ORDER=7 timeout -k 10 300 $B --sessions 1048576 > $OUT/h1m_o7.log 2>&1 && echo h-o7-ok && \
timeout -k 10 300 $B --sessions 1048576 > $OUT/h1m.log 2>&1 && echo h1m-ok && \
timeout -k 10 300 $B > $OUT/h4m.log 2>&1 && echo h4m-ok && \
timeout -k 10 300 python bench.py --graph --no-scalar --no-api --steps 20 --warmup 3 > $OUT/bench_graph.log 2>&1 && echo graph-ok
rc=$?
rm -rf $OUT/kt
tail -1 $OUT/pytest.log
for f in c2_fused c2_unfused c2_w3; do echo $f; tail -1 $OUT/$f.log | cut -c1-200; done
for f in h1m_o7 h1m h4m bench_graph; do echo $f; tail -1 $OUT/$f.log | cut -c1-200; done
exit $rc
