#!/bin/bash
# round 3: top-k selection experiments (timing-only variants) at Q = 1024 on Gaussian data,
# the instrumented append / compaction counts, and the C3 tower GEMM baseline
cd "$(dirname "$0")/.."
export TMPDIR=/tmp GAUSS=1 PREC=6
run() { echo "+ $*"; "$@"; local rc=$?; if [ $rc -ne 0 ]; then echo "FAILED rc=$rc"; exit $rc; fi; }
for rep in 1 2; do
  for v in cur nosel tau1 tau4; do
    if [ $v = cur ]; then unset RECSYS_HIP_LIB; else export RECSYS_HIP_LIB=tools/_exp_topk_$v.so; fi
    echo "== $v"
    run timeout -k 10 120 python tools/microbench_topk.py 12500000 100 1024
  done
done
for v in stats statstau1; do
  export RECSYS_HIP_LIB=tools/_exp_topk_$v.so
  echo "== $v"
  run timeout -k 10 120 python tools/topk_stats.py 12500000 100 64,1024
done
unset RECSYS_HIP_LIB
run timeout -k 10 120 python tools/microbench_towers.py
