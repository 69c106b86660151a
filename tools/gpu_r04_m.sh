#!/bin/bash
# round 4: bench lines with the pre-rolled gather / roofline brackets (c3 graphed, c5 eager)
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
for c in c3 c5; do
  timeout -k 10 300 python -u bench.py --config $c --extras off --no-cpu-baseline --no-f32-compare --steps 30 \
      -o gpurun_out/r04_m_$c.json > gpurun_out/r04_m_$c.log 2>&1 || exit $?
  python3 -c "
import json; d=json.load(open('gpurun_out/r04_m_$c.json')); r=d['roofline']
print('$c', d['ms_per_step'], r['frac'], r['avg_launch_ms'], json.dumps(r.get('gather',{}).get('in_step'))[:300])"
done
