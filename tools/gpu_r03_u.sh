#!/bin/bash
# round 3 (session 2): two-phase top-k -- parity (new tests, C4 shard, existing top-k tests), then
# Q = 1024 timing A/B over the sample fraction and against the single-pass list scan
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_topk_two_phase.py tests/test_gpu_c4_shard.py -x -v --timeout 300 \
    --timeout-method thread > gpurun_out/r03_u_tests.log 2>&1
rc=$?; echo "tp tests rc=$rc"; tail -3 gpurun_out/r03_u_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -k topk \
    > gpurun_out/r03_u_tests2.log 2>&1
rc=$?; echo "topk tests rc=$rc"; tail -2 gpurun_out/r03_u_tests2.log
if [ $rc -ne 0 ]; then exit $rc; fi
for v in "RS_TOPK_TWO_PHASE=0" "RS_TOPK_SAMPLE_DIV=16" "RS_TOPK_SAMPLE_DIV=8" "RS_TOPK_SAMPLE_DIV=32" "RS_TOPK_SAMPLE_DIV=64"; do
  env $v GAUSS=1 PREC=6 timeout -k 10 200 python -u tools/microbench_topk.py 12500000 100 1024 \
      > gpurun_out/r03_u_mb_${v}.log 2>&1 || exit $?
  echo "$v: $(grep 'Q= 1024' gpurun_out/r03_u_mb_${v}.log)"
done
