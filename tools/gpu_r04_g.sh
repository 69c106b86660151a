#!/bin/bash
# round 4: kept scores in the accumulator-native layout + fence-free tickets: the in-batch /
# model tests, then the c3 line (no profiler) and its kernel trace
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_inbatch_dedup.py \
    tests/test_gpu_c3_dedup_at_size.py tests/test_gpu_production_sizes.py tests/test_gpu_model.py \
    -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r04_g_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -4 gpurun_out/r04_g_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --extras off --no-cpu-baseline --no-f32-compare --steps 30 \
    -o gpurun_out/r04_g_c3.json > gpurun_out/r04_g_c3.log 2>&1 || exit $?
python3 -c "import json; d=json.load(open('gpurun_out/r04_g_c3.json')); print('c3', d['ms_per_step'], d['value'], d['roofline']['frac'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r04g -o g -- \
    python3 bench.py --extras off --no-cpu-baseline --no-f32-compare --steps 20 --warmup 3 > gpurun_out/r04_g_prof.log 2>&1 || exit $?
f=$(find gpurun_out/prof_r04g -name "*results.db" | head -1); python3 tools/rocpd_stats.py $f gpurun_out/r04_g_kstats.csv 30 > gpurun_out/r04_g_kstats.txt 2>&1; head -12 gpurun_out/r04_g_kstats.txt
