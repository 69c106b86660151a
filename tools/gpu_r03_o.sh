#!/bin/bash
# round 3: weight-gradient GEMM with fused column sums -- GEMM tests, the c3 line + kernel stats, c5
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread \
    -k "gemm or tower or mlp or dcn" > gpurun_out/r03_gemm_tests4.log 2>&1
rc=$?; echo "gemm tests rc=$rc"
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r03_c3cs -o run -- \
    python3 bench.py --config c3 --steps 20 --warmup 3 --no-cpu-baseline --no-f32-compare --extras off \
    -o gpurun_out/prof_r03_c3cs.json > gpurun_out/prof_r03_c3cs.log 2>&1 || exit $?
echo "prof ok"
timeout -k 10 300 python -u bench.py --config c3 --steps 30 --warmup 5 --no-cpu-baseline --extras off --no-f32-compare \
    -o gpurun_out/r03_c3_cs.json > gpurun_out/r03_c3_cs.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --config c5 --steps 10 --warmup 3 --no-cpu-baseline \
    -o gpurun_out/r03_c5_cs.json > gpurun_out/r03_c5_cs.log 2>&1 || exit $?
echo "bench ok"
