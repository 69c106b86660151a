#!/bin/bash
# round 3 (session 2): stream overlap A/B -- retrieval loss on a side stream beside the ranking
# branch, dense Adagrad beside the sparse one (RS_OVERLAP_RETRIEVAL / RS_OVERLAP_OPTIM), c2 (graphed)
# and c3 (eager), alternating; then the graphed-vs-eager bitwise tests under the default
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    -k "graphed or bitwise or c2 or reference_dims or multitask or deterministic" > gpurun_out/r03_v_tests.log 2>&1
rc=$?; echo "overlap tests rc=$rc"; tail -3 gpurun_out/r03_v_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
for i in 1 2; do
  for v in "RS_OVERLAP_RETRIEVAL=0 RS_OVERLAP_OPTIM=0" "RS_OVERLAP_RETRIEVAL=1 RS_OVERLAP_OPTIM=1" "RS_OVERLAP_RETRIEVAL=0 RS_OVERLAP_OPTIM=1"; do
    tag=$(echo $v | tr ' =' '__')
    env $v timeout -k 10 200 python -u bench.py --config c2 --steps 300 --warmup 20 --no-cpu-baseline --extras off \
        --no-f32-compare -o gpurun_out/r03_v_c2_${tag}_$i.json > gpurun_out/r03_v_c2_${tag}_$i.log 2>&1 || exit $?
    echo "c2 $v: $(python3 -c "import json;d=json.load(open('gpurun_out/r03_v_c2_${tag}_$i.json'));print(d['ms_per_step'])")"
  done
  for v in "RS_OVERLAP_RETRIEVAL=0" "RS_OVERLAP_RETRIEVAL=1"; do
    tag=$(echo $v | tr ' =' '__')
    env $v timeout -k 10 200 python -u bench.py --config c3 --steps 30 --warmup 5 --no-cpu-baseline --extras off \
        --no-f32-compare -o gpurun_out/r03_v_c3_${tag}_$i.json > gpurun_out/r03_v_c3_${tag}_$i.log 2>&1 || exit $?
    echo "c3 $v: $(python3 -c "import json;d=json.load(open('gpurun_out/r03_v_c3_${tag}_$i.json'));print(d['ms_per_step'], d['roofline']['frac'])")"
  done
done
