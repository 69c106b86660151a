#!/bin/bash
# round 4: the stack kernels loading weight fragments two chunks ahead at 16 rows: stack tests, c2 lines
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q --timeout 120 --timeout-method thread \
    -k "mlp or tower" > gpurun_out/r04_nb3_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -1 gpurun_out/r04_nb3_tests.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2 3; do
  timeout -k 10 300 python -u bench.py --config c2 --extras off --no-cpu-baseline --no-f32-compare --steps 100 \
      -o gpurun_out/r04_nb3_c2_$i.json > gpurun_out/r04_nb3_c2_$i.log 2>&1 || exit $?
  python3 -c "import json; d=json.load(open('gpurun_out/r04_nb3_c2_$i.json')); print('c2', d['ms_per_step'], d['value'])"
done
