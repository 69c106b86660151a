#!/bin/bash
# round 4: the stack weight-gradient kernel at 64-row chunks (three workgroups per CU): the
# microbench, the stack-kernel and model tests, c2 lines with the stack kernels off / on
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 python3 tools/microbench_mlp.py > gpurun_out/r04_x_mb.log 2>&1 || exit 1
grep "us per call" gpurun_out/r04_x_mb.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q --timeout 120 --timeout-method thread \
    -k "mlp or tower or gemm_group" > gpurun_out/r04_x_tests.log 2>&1
rc=$?; echo "mlp tests rc=$rc"; tail -1 gpurun_out/r04_x_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u -m pytest tests/test_gpu_model.py tests/test_gpu_dcn2.py -m gpu -x -q --timeout 300 \
    --timeout-method thread > gpurun_out/r04_x_tests_model.log 2>&1
rc=$?; echo "model tests rc=$rc"; tail -1 gpurun_out/r04_x_tests_model.log; [ $rc -eq 0 ] || exit $rc
for v in 0 16384 0 16384; do
  RS_MLP_FUSED_MAX_M=$v timeout -k 10 300 python -u bench.py --config c2 --extras off --no-cpu-baseline \
      --no-f32-compare --steps 100 -o gpurun_out/r04_x_c2_$v.json > gpurun_out/r04_x_c2_$v.log 2>&1 || exit $?
  python3 -c "import json; d=json.load(open('gpurun_out/r04_x_c2_$v.json')); print('c2 fused<=$v', d['ms_per_step'], d['value'])"
done
