#!/bin/bash
# round 4: the small-batch in-batch pair's split target (RS_IB_SPLIT_TARGET) at C2
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in 512 256 1024 512 256 1024; do
  RS_IB_SPLIT_TARGET=$v timeout -k 10 300 python -u bench.py --config c2 --extras off --no-cpu-baseline \
      --no-f32-compare --steps 100 -o gpurun_out/r04_split_c2_$v.json > gpurun_out/r04_split_c2_$v.log 2>&1 || exit $?
  python3 -c "import json; d=json.load(open('gpurun_out/r04_split_c2_$v.json')); print('c2 target=$v', d['ms_per_step'], d['value'])"
done
