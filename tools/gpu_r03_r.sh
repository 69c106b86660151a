#!/bin/bash
# round 3: skinny GEMM with batched epilogue loads -- GEMM tests, towers A/B (generic epilogue vs
# EK variants, wide-mask dX on skinny), c3 line
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_inbatch_dedup.py -x -q --timeout 120 \
    --timeout-method thread -k "gemm or tower or mlp or skinny or dedup or unique" > gpurun_out/r03_gemm_tests5.log 2>&1
rc=$?; echo "gemm tests rc=$rc"
if [ $rc -ne 0 ]; then exit $rc; fi
RS_SKINNY_WIDE_MASK=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 \
    --timeout-method thread -k "skinny or tower_group or gemm_group" > gpurun_out/r03_gemm_tests5_wm.log 2>&1
rc=$?; echo "gemm tests wm rc=$rc"
if [ $rc -ne 0 ]; then exit $rc; fi
for i in 1 2; do
  RS_SKINNY_EPI_GENERIC=1 timeout -k 10 120 python -u tools/microbench_towers.py > gpurun_out/r03_skg_$i.log 2>&1 || exit $?
  timeout -k 10 120 python -u tools/microbench_towers.py > gpurun_out/r03_skn_$i.log 2>&1 || exit $?
  RS_SKINNY_WIDE_MASK=1 timeout -k 10 120 python -u tools/microbench_towers.py > gpurun_out/r03_skw_$i.log 2>&1 || exit $?
done
timeout -k 10 300 python -u bench.py --config c3 --steps 30 --warmup 5 --no-cpu-baseline --extras off --no-f32-compare \
    -o gpurun_out/r03_c3_ek.json > gpurun_out/r03_c3_ek.log 2>&1 || exit $?
RS_SKINNY_WIDE_MASK=1 timeout -k 10 300 python -u bench.py --config c3 --steps 30 --warmup 5 --no-cpu-baseline \
    --extras off --no-f32-compare -o gpurun_out/r03_c3_ekw.json > gpurun_out/r03_c3_ekw.log 2>&1 || exit $?
echo done
