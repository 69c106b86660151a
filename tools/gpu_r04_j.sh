#!/bin/bash
# round 4: onesweep vs rocprim's merge-path radix sort (id plans, sparse Adagrad): tests, then
# c3 eager / c5 / c3 graphed lines alternating RS_SORT_MERGE (onesweep only outside capture)
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_inbatch_dedup.py tests/test_gpu_kernels.py tests/test_gpu_model.py \
    tests/test_gpu_multirank.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r04_j_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r04_j_tests.log; [ $rc -eq 0 ] || exit $rc
for c in c3 c5 c3g; do for m in 0 1 0 1; do
  case $c in c3) a="--config c3 --eager";; c3g) a="--config c3";; *) a="--config $c";; esac
  RS_SORT_MERGE=$m timeout -k 10 300 python -u bench.py $a --extras off --no-cpu-baseline --no-f32-compare \
      --steps 40 -o gpurun_out/r04_j_${c}_$m.json > gpurun_out/r04_j_${c}_$m.log 2>&1 || exit $?
  python3 -c "import json; d=json.load(open('gpurun_out/r04_j_${c}_$m.json')); print('$c merge=$m', d['ms_per_step'], d['value'], d['roofline']['frac'])"
done; done
