#!/bin/bash
# Alternating A/B of librecsys_hip.so variants on the C3 bench line (3 rounds, 30 timed steps,
# no extras): per round and variant the step time, roofline fraction and the in-batch entry points'
# launch times. Usage: tools/gpu_ab_c3.sh lib1.so lib2.so ...   (results: gpurun_out/abc3/)
# A lib named nows*.so runs with RS_GEMM_NO_WS=1 (an -DRS_EXPERIMENTS build of gemm.hip).
set -e
out=gpurun_out/abc3
mkdir -p $out
for round in 1 2 3; do
  for lib in "$@"; do
    tag=$(basename $lib .so)
    env=""; case $tag in nows*) env="RS_GEMM_NO_WS=1" ;; esac
    env $env RECSYS_HIP_LIB=$lib timeout -k 10 180 python bench.py --config c3 --steps 30 --warmup 3 --no-cpu-baseline \
      --no-f32-compare --extras off > $out/${tag}_$round.json 2> $out/${tag}_$round.err
    python - "$out/${tag}_$round.json" "$tag" "$round" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d["roofline"]
print(f"{sys.argv[3]} {sys.argv[2]:24s} {d['ms_per_step']:7.3f} ms/step  frac {r['frac']}  {r.get('per_entry_ms')}", flush=True)
PY
  done
done
