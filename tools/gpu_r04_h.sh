#!/bin/bash
# round 4: c3 step modes A/B: eager with host-read dedup counts, eager with device counts, graphed
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {  # tag, env, args
  env $2 timeout -k 10 300 python -u bench.py --extras off --no-cpu-baseline --no-f32-compare --steps 40 $3 \
      -o gpurun_out/r04_h_$1.json > gpurun_out/r04_h_$1.log 2>&1 || return $?
  python3 -c "import json; d=json.load(open('gpurun_out/r04_h_$1.json')); print('$1', d['ms_per_step'], d['value'], d['roofline']['frac'])"
}
for i in 1 2; do
  run host$i "RS_INBATCH_DEDUP_DEVICE=0" "" || exit $?
  run dev$i "RS_INBATCH_DEDUP_DEVICE=1" "" || exit $?
  run graph$i "RS_INBATCH_DEDUP_DEVICE=0" "--graph" || exit $?
done
