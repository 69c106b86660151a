#!/bin/bash
# round 3: wide-mask dX on the skinny kernel inside the c3 step, alternating A/B (same box)
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
for i in 1 2; do
  RS_SKINNY_WIDE_MASK=1 timeout -k 10 300 python -u bench.py --config c3 --steps 30 --warmup 5 --no-cpu-baseline \
      --extras off --no-f32-compare -o gpurun_out/r03_c3_w$i.json > gpurun_out/r03_c3_w$i.log 2>&1 || exit $?
  timeout -k 10 300 python -u bench.py --config c3 --steps 30 --warmup 5 --no-cpu-baseline --extras off \
      --no-f32-compare -o gpurun_out/r03_c3_n$i.json > gpurun_out/r03_c3_n$i.log 2>&1 || exit $?
done
echo done
SHAPES="c3 tower fwd" KPAT=gemm_skinny PRECS=6 bash tools/gpu_pmc_gemm_stalls.sh > gpurun_out/r03_pmc_skinny.txt 2>&1 || exit $?
echo pmc done
