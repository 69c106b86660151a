#!/bin/bash
# round 3 (session 2): 8-wave threshold scan (RS_TOPK_THR_W8=1; =2 with 64-row tiles) vs the 4-wave default
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
o=gpurun_out/r03_w8_ab.txt; : > $o
for m in 1 2; do
  RS_TOPK_THR_W8=$m PREC=6 timeout -k 10 200 python -u tools/microbench_topk.py 12500000 100 1024 >> $o 2>&1 || exit $?
done
for i in 1 2; do
  for m in 0 1 2; do
    echo "== w8=$m $i" >> $o
    RS_TOPK_THR_W8=$m GAUSS=1 PREC=6 timeout -k 10 200 python -u tools/microbench_topk.py 12500000 100 1024 >> $o 2>&1 || exit $?
  done
done
grep -v amdgpu.ids $o
