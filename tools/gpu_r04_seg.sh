#!/bin/bash
# round 4: the sparse update's LDS sort one workgroup per table: the sort tests, c2 lines and the
# c2 kernel stats
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q --timeout 120 --timeout-method thread \
    -k "sparse" > gpurun_out/r04_seg_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -1 gpurun_out/r04_seg_tests.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --config c2 --extras off --no-cpu-baseline --no-f32-compare --steps 100 \
      -o gpurun_out/r04_seg_c2_$i.json > gpurun_out/r04_seg_c2_$i.log 2>&1 || exit $?
  python3 -c "import json; d=json.load(open('gpurun_out/r04_seg_c2_$i.json')); print('c2', d['ms_per_step'], d['value'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_seg -o c2 -- python3 bench.py --config c2 \
    --extras off --no-cpu-baseline --no-f32-compare --steps 20 --warmup 3 -o gpurun_out/r04_seg_prof.json \
    > gpurun_out/r04_seg_prof.log 2>&1 || exit $?
f=$(find gpurun_out/prof_seg -name "*results.db" | head -1)
python3 tools/rocpd_stats.py $f gpurun_out/r04_seg_c2_kernel_stats.csv 60 > gpurun_out/r04_seg_c2_kernel_stats.txt 2>&1
rm -rf gpurun_out/prof_seg
head -14 gpurun_out/r04_seg_c2_kernel_stats.txt | cut -c1-130
