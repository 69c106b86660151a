#!/bin/bash
# round 3: skinny GEMM (4-wave workgroups) tests + tower A/B, then the multi-rank tests
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread \
    -k "skinny or gemm_group or tower_group or gemm" > gpurun_out/r03_gemm_tests2.log 2>&1
rc=$?; echo "gemm tests rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for rep in 1 2; do
  RS_GEMM_NO_SKINNY=1 timeout -k 10 120 python tools/microbench_towers.py > gpurun_out/r03_towers2_old_$rep.log 2>&1 || exit $?
  timeout -k 10 120 python tools/microbench_towers.py > gpurun_out/r03_towers2_new_$rep.log 2>&1 || exit $?
done
echo "towers ok"
timeout -k 10 600 python -u -m pytest tests/test_gpu_multirank.py -v -s --timeout 300 --timeout-method thread > gpurun_out/r03_multirank2.log 2>&1
echo "multirank rc=$?"
