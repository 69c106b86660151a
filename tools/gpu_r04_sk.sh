#!/bin/bash
# round 4: the large-batch tower GEMMs reading weight fragment images (RS_SKINNY_IMG): the bitwise
# test and the stack tests, then c3 lines with images off / on
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q --timeout 120 --timeout-method thread \
    -k "mlp or tower or gemm_group or skinny" > gpurun_out/r04_sk_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -1 gpurun_out/r04_sk_tests.log; [ $rc -eq 0 ] || exit $rc
for v in 0 1 0 1; do
  RS_SKINNY_IMG=$v timeout -k 10 300 python -u bench.py --config c3 --extras off --no-cpu-baseline --no-f32-compare \
      --steps 30 -o gpurun_out/r04_sk_c3_$v.json > gpurun_out/r04_sk_c3_$v.log 2>&1 || exit $?
  python3 -c "import json; d=json.load(open('gpurun_out/r04_sk_c3_$v.json')); print('c3 img=$v', d['ms_per_step'], d['value'], d['roofline']['frac'])"
done
RS_SKINNY_IMG=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_sk -o c3 -- python3 bench.py \
    --extras off --no-cpu-baseline --no-f32-compare --steps 20 --warmup 3 -o gpurun_out/r04_sk_prof.json \
    > gpurun_out/r04_sk_prof.log 2>&1 || exit $?
f=$(find gpurun_out/prof_sk -name "*results.db" | head -1)
python3 tools/rocpd_stats.py $f gpurun_out/r04_sk_c3_kernel_stats.csv 60 > gpurun_out/r04_sk_c3_kernel_stats.txt 2>&1
rm -rf gpurun_out/prof_sk
grep -E "skinny|gemm_x3|mlp_image" gpurun_out/r04_sk_c3_kernel_stats.txt | cut -c1-130
