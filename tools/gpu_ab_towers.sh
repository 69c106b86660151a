#!/bin/bash
# Alternating A/B of librecsys_hip.so variants on the C3 tower layers (tools/microbench_towers.py,
# 2 rounds). Usage: tools/gpu_ab_towers.sh lib1.so lib2.so ...   (results: gpurun_out/abtw/)
# A lib named nows*.so runs with RS_GEMM_NO_WS=1 (an -DRS_EXPERIMENTS build of gemm.hip).
set -e
out=gpurun_out/abtw
mkdir -p $out
for round in 1 2; do
  for lib in "$@"; do
    tag=$(basename $lib .so)
    env=""; case $tag in nows*) env="RS_GEMM_NO_WS=1" ;; esac
    env $env RECSYS_HIP_LIB=$lib timeout -k 10 120 python tools/microbench_towers.py 65536 > $out/${tag}_$round.log 2>&1
    echo "$round $tag $(grep total $out/${tag}_$round.log)"
  done
done
