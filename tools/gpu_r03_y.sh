#!/bin/bash
# (timing split of the ratio choice; the tests of tools/gpu_r03_x.sh first)
# round 3 (session 2): bound-first top-k timing split -- the threshold scans alone (+inf bound,
# RS_TOPK_EXP_TH_INF: no candidates, wrong lists) against the default and the list scan; kernel trace
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
for i in 1; do
for v in "RS_TOPK_TWO_PHASE=0" "RS_TOPK_RANGE_RATIO=4" "RS_TOPK_RANGE_RATIO=8" "RS_TOPK_EXP_TH_INF=1"; do
  env $v GAUSS=1 PREC=6 timeout -k 10 200 python -u tools/microbench_topk.py 12500000 100 1024 \
      > gpurun_out/r03_y_mb_${v}_$i.log 2>&1 || exit $?
  echo "$v: $(grep 'Q= 1024' gpurun_out/r03_y_mb_${v}_$i.log)"
done
done
GAUSS=1 PREC=6 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_tp3 -o tp -- \
    python3 tools/microbench_topk.py 12500000 100 1024 > gpurun_out/r03_y_tp.log 2>&1 || exit $?
f=$(find gpurun_out/prof_tp3 -name '*kernel_stats.csv' | head -1); python3 tools/kstats.py $f 4
