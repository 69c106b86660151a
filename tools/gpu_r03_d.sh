#!/bin/bash
# round 3: skinny-GEMM tests + tower A/B, top-k selection experiments, multi-rank tests, bench lines
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread \
    -k "skinny or gemm_group or tower_group or gemm" > gpurun_out/r03_gemm_tests.log 2>&1
rc=$?; echo "gemm tests rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
if [ $rc -ne 0 ]; then export RS_GEMM_NO_SKINNY=1; fi
for rep in 1 2; do
  RS_GEMM_NO_SKINNY=1 timeout -k 10 120 python tools/microbench_towers.py > gpurun_out/r03_towers_old_$rep.log 2>&1 || exit $?
  timeout -k 10 120 python tools/microbench_towers.py > gpurun_out/r03_towers_new_$rep.log 2>&1 || exit $?
done
echo "towers ok"
# top-k variants (timing only) and the instrumented counts
(
  export GAUSS=1 PREC=6
  for rep in 1 2; do
    for v in cur nosel tau1 tau4; do
      if [ $v = cur ]; then unset RECSYS_HIP_LIB; else export RECSYS_HIP_LIB=tools/_exp_topk_$v.so; fi
      echo "== $v"
      timeout -k 10 120 python tools/microbench_topk.py 12500000 100 1024 || exit $?
    done
  done
  for v in stats statstau1; do
    export RECSYS_HIP_LIB=tools/_exp_topk_$v.so
    echo "== $v"
    timeout -k 10 120 python tools/topk_stats.py 12500000 100 64,1024 || exit $?
  done
) > gpurun_out/r03_topk_exp.log 2>&1 || { echo "topk exp failed"; exit 1; }
echo "topk ok"
bash tools/gpu_r03_b.sh
