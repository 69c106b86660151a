#!/bin/bash
# round 4: every stack node's weight images of a step in one launch (RS_MLP_PREPARE): model / stack
# tests, c2 lines off / on
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_model.py tests/test_gpu_kernels.py tests/test_gpu_inbatch_dedup.py \
    -m gpu -x -q --timeout 300 --timeout-method thread -k "model or step or mlp or tower or graph or golden" \
    > gpurun_out/r04_prep_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -1 gpurun_out/r04_prep_tests.log; [ $rc -eq 0 ] || exit $rc
for v in 0 1 0 1; do
  RS_MLP_PREPARE=$v timeout -k 10 300 python -u bench.py --config c2 --extras off --no-cpu-baseline --no-f32-compare \
      --steps 100 -o gpurun_out/r04_prep_c2_$v.json > gpurun_out/r04_prep_c2_$v.log 2>&1 || exit $?
  python3 -c "import json; d=json.load(open('gpurun_out/r04_prep_c2_$v.json')); print('c2 prepare=$v', d['ms_per_step'], d['value'])"
done
