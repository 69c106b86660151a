#!/bin/bash
# round 3: top-k A/B (round-2 kernel vs current vs deferred compaction), then the PMC traffic passes
# and the per-config rocprofv3 kernel statistics of the bench
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
(
  export GAUSS=1 PREC=6
  for rep in 1 2; do
    for v in cur old defer; do
      if [ $v = cur ]; then unset RECSYS_HIP_LIB; else export RECSYS_HIP_LIB=tools/_exp_topk_$v.so; fi
      echo "== $v"
      timeout -k 10 120 python tools/microbench_topk.py 12500000 100 1024 || exit $?
    done
  done
) > gpurun_out/r03_topk_ab2.log 2>&1 || { echo "topk ab failed"; exit 1; }
echo "topk ab ok"
bash tools/gpu_r03_pmc.sh > gpurun_out/r03_pmc.log 2>&1 || { echo "pmc failed"; exit 1; }
echo "pmc ok"
for c in c3 c5 c4; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r03_$c -o run -- \
      python3 bench.py --config $c --steps 10 --warmup 3 --no-cpu-baseline --no-f32-compare --extras off \
      -o gpurun_out/prof_r03_$c.json > gpurun_out/prof_r03_$c.log 2>&1 || { echo "prof $c failed"; exit 1; }
done
echo "prof ok"
