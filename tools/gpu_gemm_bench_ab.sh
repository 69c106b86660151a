#!/bin/bash
# GEMM variant A/B (tools/_exp_gemm_<v>.so in VARS): c3 tower shapes, then c3 / c2 bench steps, twice
SHAPES=c3 VARS="${VARS}" bash tools/gpu_gemm_exp.sh > gpurun_out/gemm_ab.log 2>&1
for rep in 1 2; do
for v in cur ${VARS}; do
  if [ $v = cur ]; then unset RECSYS_HIP_LIB; else export RECSYS_HIP_LIB=tools/_exp_gemm_$v.so; fi
  timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-f32-compare -o gpurun_out/ab_c3_$v.json > /dev/null 2>&1 || exit 1
  timeout -k 10 300 python bench.py --config c2 --steps 100 --warmup 5 --no-cpu-baseline -o gpurun_out/ab_c2_$v.json > /dev/null 2>&1 || exit 1
  python -c "import json;[print('$v', c, json.load(open(f'gpurun_out/ab_{c}_$v.json'))['ms_per_step']) for c in ('c3','c2')]"
done
done
