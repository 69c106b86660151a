#!/bin/bash
# round 4: slab reductions with two rounds of loads in flight: the reduction / defer / model tests,
# c3 lines and the c3 kernel stats
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_model.py -m gpu -x -q --timeout 300 \
    --timeout-method thread > gpurun_out/r04_slab_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -1 gpurun_out/r04_slab_tests.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --config c3 --extras off --no-cpu-baseline --no-f32-compare --steps 40 \
      -o gpurun_out/r04_slab_c3_$i.json > gpurun_out/r04_slab_c3_$i.log 2>&1 || exit $?
  python3 -c "import json; d=json.load(open('gpurun_out/r04_slab_c3_$i.json')); print('c3', d['ms_per_step'], d['value'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_slab -o c3 -- python3 bench.py \
    --extras off --no-cpu-baseline --no-f32-compare --steps 20 --warmup 3 -o gpurun_out/r04_slab_prof.json \
    > gpurun_out/r04_slab_prof.log 2>&1 || exit $?
f=$(find gpurun_out/prof_slab -name "*results.db" | head -1)
python3 tools/rocpd_stats.py $f gpurun_out/r04_slab_c3_kernel_stats.csv 60 > gpurun_out/r04_slab_c3_kernel_stats.txt 2>&1
rm -rf gpurun_out/prof_slab
grep -E "slab|inbatch_row_m16" gpurun_out/r04_slab_c3_kernel_stats.txt | cut -c1-130
