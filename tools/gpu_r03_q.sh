#!/bin/bash
# round 3: skinny GEMM variants for the wide masked dX (A/B in one call) + torch-op census of c3
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in base wm nw8 both; do
  case $v in
    base) env_set="";;
    wm) env_set="RS_SKINNY_WIDE_MASK=1";;
    nw8) env_set="RS_SKINNY_NT16_NW8=1";;
    both) env_set="RS_SKINNY_WIDE_MASK=1 RS_SKINNY_NT16_NW8=1";;
  esac
  env $env_set timeout -k 10 120 python -u tools/microbench_towers.py > gpurun_out/r03_sk_$v.log 2>&1 || exit $?
done
timeout -k 10 200 python -u tools/prof_torch_ops.py c3 > gpurun_out/r03_torchops_c3.txt 2>&1 || exit $?
echo done
