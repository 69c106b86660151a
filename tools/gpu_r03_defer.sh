#!/bin/bash
# round 3 (session 2): deferred gradient reductions -- tests, then c2 / c3 / c5 A/B
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
    -k "deferred_reductions_each or deferred or graphed or model or multitask or train or c2 or production or dcn2 or golden or multirank" \
    > gpurun_out/r03_defer_tests.log 2>&1
rc=$?; echo "defer tests rc=$rc"; tail -3 gpurun_out/r03_defer_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
for i in 1 2; do
  timeout -k 10 200 python -u bench.py --config c2 --steps 300 --warmup 20 --no-cpu-baseline --extras off \
      --no-f32-compare -o gpurun_out/r03_defer_c2_$i.json > gpurun_out/r03_defer_c2_$i.log 2>&1 || exit $?
  python3 -c "import json;d=json.load(open('gpurun_out/r03_defer_c2_$i.json'));print('c2', d['ms_per_step'], d['value'])"
  timeout -k 10 300 python -u bench.py --config c3 --steps 50 --warmup 5 --no-cpu-baseline --extras off \
      --no-f32-compare -o gpurun_out/r03_defer_c3_$i.json > gpurun_out/r03_defer_c3_$i.log 2>&1 || exit $?
  python3 -c "import json;d=json.load(open('gpurun_out/r03_defer_c3_$i.json'));print('c3', d['ms_per_step'], d['value'])"
done
timeout -k 10 300 python -u bench.py --config c5 --steps 20 --warmup 3 --no-cpu-baseline --extras off \
    --no-f32-compare -o gpurun_out/r03_defer_c5.json > gpurun_out/r03_defer_c5.log 2>&1 || exit $?
python3 -c "import json;d=json.load(open('gpurun_out/r03_defer_c5.json'));print('c5', d['ms_per_step'], d['value'])"
