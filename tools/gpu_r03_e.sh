#!/bin/bash
# round 3: deferred top-k compaction -- parity (dyadic bit-exact tests incl. the 12.5M shard), A/B
# against the previous kernel, instrumented counts; then the step-by-step multi-rank tests
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_c4_shard.py -x -q --timeout 200 \
    --timeout-method thread -k "topk or c4" > gpurun_out/r03_topk_tests.log 2>&1
rc=$?; echo "topk tests rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
(
  export GAUSS=1 PREC=6
  for rep in 1 2 3; do
    for v in new old; do
      if [ $v = new ]; then unset RECSYS_HIP_LIB; else export RECSYS_HIP_LIB=tools/_exp_topk_$v.so; fi
      echo "== $v"
      timeout -k 10 120 python tools/microbench_topk.py 12500000 100 1,64,1024 || exit $?
    done
  done
  export RECSYS_HIP_LIB=tools/_exp_topk_stats.so
  echo "== stats (new)"
  timeout -k 10 120 python tools/topk_stats.py 12500000 100 64,1024 || exit $?
) > gpurun_out/r03_topk_ab.log 2>&1 || { echo "topk ab failed"; exit 1; }
echo "topk ab ok"
timeout -k 10 600 python -u -m pytest tests/test_gpu_multirank.py -v --timeout 300 --timeout-method thread > gpurun_out/r03_multirank.log 2>&1
echo "multirank rc=$?"
