#!/bin/bash
# round 4: the in-step gather on uniform ids, id-ordered vs batch-ordered (RS_GATHER_ORDERED), c3 step
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
for o in 1 0 1 0; do
  RS_BENCH_IDS=uniform RS_GATHER_ORDERED=$o timeout -k 10 300 python -u bench.py --extras off --no-cpu-baseline \
      --no-f32-compare --steps 10 -o gpurun_out/r04_p_u$o.json > gpurun_out/r04_p_u$o.log 2>&1 || exit $?
  python3 -c "
import json; d=json.load(open('gpurun_out/r04_p_u$o.json')); g=d['roofline']['gather']
print('uniform ordered=$o', d['ms_per_step'], g['in_step']['frac'], g['in_step']['avg_launch_ms'], g['uniform_standalone']['frac'])"
done
for o in 1 0; do
  RS_GATHER_ORDERED=$o timeout -k 10 300 python -u bench.py --extras off --no-cpu-baseline \
      --no-f32-compare --steps 30 -o gpurun_out/r04_p_z$o.json > gpurun_out/r04_p_z$o.log 2>&1 || exit $?
  python3 -c "
import json; d=json.load(open('gpurun_out/r04_p_z$o.json')); g=d['roofline']['gather']
print('zipf ordered=$o', d['ms_per_step'], g['in_step']['frac'], g['in_step']['avg_launch_ms'])"
done
