#!/bin/bash
# A/B of librecsys_hip.so variants (RECSYS_HIP_LIB) in one box: the in-batch precision diagnostic
# and short c2 / c3 bench lines per variant, alternated twice. Usage: tools/gpu_r05_ab.sh lib1 lib2 ...
set -e
out=gpurun_out/ab
mkdir -p $out
for round in 1 2; do
  for lib in "$@"; do
    tag=$(basename $lib .so)
    if [ $round = 1 ]; then
      RECSYS_HIP_LIB=$lib timeout -k 10 120 python tools/diag_inbatch_prec.py > $out/diag_$tag.log 2>&1
    fi
    RECSYS_HIP_LIB=$lib timeout -k 10 180 python bench.py --config c3 --steps 30 --warmup 3 --no-cpu-baseline --no-f32-compare --extras off > $out/c3_${tag}_$round.json 2> $out/c3_${tag}_$round.err
    RECSYS_HIP_LIB=$lib timeout -k 10 180 python bench.py --config c2 --steps 200 --warmup 10 --no-cpu-baseline --no-f32-compare --extras off > $out/c2_${tag}_$round.json 2> $out/c2_${tag}_$round.err
    echo "$round $tag done"
  done
done
