#!/bin/bash
# round 3: deduplicated in-batch pair tests; skinny-GEMM gate tests; the c2 line; the default line
# with and without the deduplicated pair
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_inbatch_dedup.py -x -v --timeout 120 --timeout-method thread \
    > gpurun_out/r03_dedup_tests.log 2>&1
rc=$?; echo "dedup tests rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread \
    -k "skinny or gemm" > gpurun_out/r03_gemm_tests3.log 2>&1
rc=$?; echo "gemm tests rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py --config c2 --steps 100 --warmup 5 --no-cpu-baseline -o gpurun_out/r03_c2b.json \
    > gpurun_out/r03_c2b.log 2>&1 || exit $?
echo "c2 ok"
timeout -k 10 300 python -u bench.py --config c3 --steps 20 --warmup 5 --no-cpu-baseline --extras off --no-f32-compare -o gpurun_out/r03_c3_dedup.json \
    > gpurun_out/r03_c3_dedup.log 2>&1 || exit $?
echo "c3 dedup ok"
RS_INBATCH_DEDUP=0 timeout -k 10 300 python -u bench.py --config c3 --steps 20 --warmup 5 --no-cpu-baseline --extras off --no-f32-compare \
    -o gpurun_out/r03_c3_full.json > gpurun_out/r03_c3_full.log 2>&1 || exit $?
echo "c3 full ok"
