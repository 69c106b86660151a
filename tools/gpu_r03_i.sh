#!/bin/bash
# round 3: top-k per-slice list length experiment (timing-only variants) + counts
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp GAUSS=1 PREC=6
(
  for rep in 1 2; do
    for v in cur kl32 kl48 kl64; do
      if [ $v = cur ]; then unset RECSYS_HIP_LIB; else export RECSYS_HIP_LIB=tools/_exp_topk_$v.so; fi
      echo "== $v"
      timeout -k 10 120 python tools/microbench_topk.py 12500000 100 1024 || exit $?
    done
  done
  for v in stats statskl32; do
    export RECSYS_HIP_LIB=tools/_exp_topk_$v.so
    echo "== $v"
    timeout -k 10 120 python tools/topk_stats.py 12500000 100 1024 || exit $?
  done
) > gpurun_out/r03_topk_kl.log 2>&1 || { echo "failed"; exit 1; }
echo ok
