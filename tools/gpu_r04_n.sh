#!/bin/bash
# round 4: one-workgroup LDS sort for small sparse updates: kernel + model tests, c2 / c3 lines, c2 stats
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_model.py tests/test_gpu_dcn2.py tests/test_gpu_multirank.py \
    tests/test_gpu_production_sizes.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r04_n_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r04_n_tests.log; [ $rc -eq 0 ] || exit $rc
for c in c2 c3; do
  timeout -k 10 300 python -u bench.py --config $c --extras off --no-cpu-baseline --no-f32-compare --steps 40 \
      -o gpurun_out/r04_n_$c.json > gpurun_out/r04_n_$c.log 2>&1 || exit $?
  python3 -c "import json; d=json.load(open('gpurun_out/r04_n_$c.json')); print('$c', d['ms_per_step'], d['value'], d['roofline']['frac'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r04n -o p -- \
    python3 bench.py --config c2 --extras off --no-cpu-baseline --no-f32-compare --steps 20 --warmup 3 > gpurun_out/r04_n_prof.log 2>&1 || exit $?
f=$(find gpurun_out/prof_r04n -name "*results.db" | head -1)
python3 tools/rocpd_stats.py $f gpurun_out/r04_n_c2_kstats.csv 60 > gpurun_out/r04_n_c2_kstats.txt 2>&1; rm -rf gpurun_out/prof_r04n
