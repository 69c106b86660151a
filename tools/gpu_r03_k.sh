#!/bin/bash
# round 3: skinny-GEMM gate (workgroup count) -- GEMM tests, the c2 line, the default line
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread \
    -k "skinny or gemm_group or tower_group or gemm" > gpurun_out/r03_gemm_tests3.log 2>&1
rc=$?; echo "gemm tests rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py --config c2 --steps 100 --warmup 5 --no-cpu-baseline -o gpurun_out/r03_c2b.json \
    > gpurun_out/r03_c2b.log 2>&1 || exit $?
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 -o gpurun_out/r03_bench3.json > gpurun_out/r03_bench3.log 2>&1 || exit $?
echo "bench ok"
