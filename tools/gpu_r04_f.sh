#!/bin/bash
# round 4: split-K slice-count A/B on the C3 tower layers (dW + db incl. the reduction) and the c3 step
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
for w in 512 256 128 64; do
  echo "== RS_SPLITK_WANT=$w"
  RS_SPLITK_WANT=$w timeout -k 10 120 python -u tools/microbench_towers.py || exit $?
done > gpurun_out/r04_f_splitk.log 2>&1
cat gpurun_out/r04_f_splitk.log | grep -v "^$"
for w in 512 128 512 128; do
  RS_SPLITK_WANT=$w timeout -k 10 200 python -u bench.py --extras off --no-cpu-baseline --no-f32-compare --steps 30 \
      -o gpurun_out/r04_f_c3_$w.json > /dev/null 2>&1 || exit $?
  python3 -c "import json; d=json.load(open('gpurun_out/r04_f_c3_$w.json')); print('want $w', d['ms_per_step'], d['roofline']['frac'])"
done
