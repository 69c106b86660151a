#!/bin/bash
# round 3 (session 2): 64- vs 96-row tiles in the 8-wave threshold scan; parity under the 64-row variant
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
o=gpurun_out/r03_w8b_ab.txt; : > $o
RS_TOPK_THR_W8=3 PREC=6 timeout -k 10 200 python -u tools/microbench_topk.py 12500000 100 1024 >> $o 2>&1 || exit $?
for i in 1 2; do
  for m in 2 3; do
    echo "== w8=$m $i" >> $o
    RS_TOPK_THR_W8=$m GAUSS=1 PREC=6 timeout -k 10 200 python -u tools/microbench_topk.py 12500000 100 1024 >> $o 2>&1 || exit $?
  done
done
grep -v amdgpu.ids $o
RS_TOPK_THR_W8=2 timeout -k 10 500 python -u -m pytest tests/test_gpu_topk_two_phase.py tests/test_gpu_c4_shard.py -x -q --timeout 300 \
    --timeout-method thread > gpurun_out/r03_w8b_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/r03_w8b_tests.log
exit $rc
