#!/bin/bash
# round 4: the wide-mask dX on the skinny kernel (RS_SKINNY_WIDE_MASK, with weight images) at C3
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in 0 1 0 1; do
  if [ $v = 1 ]; then export RS_SKINNY_WIDE_MASK=1; else unset RS_SKINNY_WIDE_MASK; fi
  timeout -k 10 300 python -u bench.py --config c3 --extras off --no-cpu-baseline --no-f32-compare --steps 40 \
      -o gpurun_out/r04_wm_c3_$v.json > gpurun_out/r04_wm_c3_$v.log 2>&1 || exit $?
  python3 -c "import json; d=json.load(open('gpurun_out/r04_wm_c3_$v.json')); print('c3 wide_mask=$v', d['ms_per_step'], d['value'])"
done
