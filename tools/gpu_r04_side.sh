#!/bin/bash
# round 4: the large-batch weight gradients on a side stream (RS_WGRAD_SIDE_STREAM): graphed-step /
# model tests with it on, then c3 lines off / on
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
RS_WGRAD_SIDE_STREAM=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_model.py tests/test_gpu_inbatch_dedup.py \
    tests/test_gpu_kernels.py -m gpu -x -q --timeout 300 --timeout-method thread \
    -k "(graph or step or model or tower or golden) and not defer" > gpurun_out/r04_side_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -1 gpurun_out/r04_side_tests.log; [ $rc -eq 0 ] || exit $rc
for v in 0 1 0 1; do
  RS_WGRAD_SIDE_STREAM=$v timeout -k 10 300 python -u bench.py --config c3 --extras off --no-cpu-baseline \
      --no-f32-compare --steps 40 -o gpurun_out/r04_side_c3_$v.json > gpurun_out/r04_side_c3_$v.log 2>&1 || exit $?
  python3 -c "import json; d=json.load(open('gpurun_out/r04_side_c3_$v.json')); print('c3 side=$v', d['ms_per_step'], d['value'])"
done
