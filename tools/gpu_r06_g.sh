#!/bin/bash
# Round 6: tests on the default build, the staggered row pass's tests on its A/B build, then C3
# kernel-statistics A/B runs (transposed col image, row stagger, setprio), then the DP rehearsals.
cd "$(dirname "$0")/.."
tag=${1:-r06g}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 400 --timeout-method thread \
    tests/test_gpu_inbatch_dedup.py tests/test_gpu_dp_sparse.py tests/test_gpu_multirank.py tests/test_gpu_model.py \
    > $out/tests.log 2>&1
rc=$?; tail -3 $out/tests.log; [ $rc -eq 0 ] || exit $rc
RECSYS_HIP_LIB=_ablibs/ib_stg1.so timeout -k 10 600 python -u -m pytest -x -v --timeout 400 --timeout-method thread \
    tests/test_gpu_inbatch_dedup.py > $out/tests_stg1.log 2>&1
rc=$?; tail -3 $out/tests_stg1.log; [ $rc -eq 0 ] || exit $rc
PROFAB_OUT=$out/ab_timg bash tools/gpu_prof_ab.sh _ablibs/ib_timg0.so _ablibs/ib_stg0.so || exit $?
PROFAB_OUT=$out/ab_stg bash tools/gpu_prof_ab.sh _ablibs/ib_stg0.so _ablibs/ib_stg1.so || exit $?
PROFAB_OUT=$out/ab_prio bash tools/gpu_prof_ab.sh _ablibs/ib_timg1.so _ablibs/ib_prio1.so || exit $?
timeout -k 10 300 python -u tools/microbench_dp_sparse.py 8 > $out/dp_sparse.log 2>&1 || exit $?
tail -1 $out/dp_sparse.log
for ex in dedupe padded; do
  timeout -k 10 300 python -u bench.py --config c3 --exchange $ex --steps 30 --no-cpu-baseline --no-f32-compare \
      -o $out/c3_exchange_$ex.json > $out/c3_exchange_$ex.log 2>&1 || exit $?
  python3 -c "import json; d=json.load(open('$out/c3_exchange_$ex.json')); print('$ex', d['ms_per_step'], d['config'].get('hipgraph'))"
done
timeout -k 10 300 python -u bench.py --config c3 --eager --extras off --steps 30 --no-cpu-baseline --no-f32-compare \
    -o $out/c3_eager.json > $out/c3_eager.log 2>&1 || exit $?
python3 -c "import json; d=json.load(open('$out/c3_eager.json')); print('eager', d['ms_per_step'])"
