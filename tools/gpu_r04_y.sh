#!/bin/bash
# round 4: the stack weight-gradient kernel at C3's batch (RS_MLP_WGRAD_MAX_M) and the whole stack
# path there (RS_MLP_FUSED_MAX_M): the paths-agree tests, then c3 lines per setting
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q --timeout 120 --timeout-method thread \
    -k "mlp or tower" > gpurun_out/r04_y_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -1 gpurun_out/r04_y_tests.log; [ $rc -eq 0 ] || exit $rc
for v in "16384 16384" "16384 65536" "65536 65536" "16384 16384" "16384 65536"; do
  set -- $v
  RS_MLP_FUSED_MAX_M=$1 RS_MLP_WGRAD_MAX_M=$2 timeout -k 10 300 python -u bench.py --config c3 --extras off \
      --no-cpu-baseline --no-f32-compare --steps 30 -o gpurun_out/r04_y_c3_$1_$2.json > gpurun_out/r04_y_c3_$1_$2.log 2>&1 || exit $?
  python3 -c "import json; d=json.load(open('gpurun_out/r04_y_c3_$1_$2.json')); print('c3 fused<=$1 wgrad<=$2', d['ms_per_step'], d['value'], d['roofline']['frac'])"
done
