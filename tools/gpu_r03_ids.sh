#!/bin/bash
# round 3 (session 2): distinct rows by id for the model's deduplicated pair -- tests, then c3 A/B
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_inbatch_dedup.py tests/test_abi.py -x -q --timeout 200 \
    --timeout-method thread > gpurun_out/r03_ids_tests.log 2>&1
rc=$?; echo "ids tests rc=$rc"; tail -3 gpurun_out/r03_ids_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
    -k "multitask or c3 or production or train or graphed or deterministic or distributed or multirank" \
    > gpurun_out/r03_ids_tests2.log 2>&1
rc=$?; echo "model tests rc=$rc"; tail -3 gpurun_out/r03_ids_tests2.log
if [ $rc -ne 0 ]; then exit $rc; fi
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --config c3 --steps 50 --warmup 5 --no-cpu-baseline --extras off \
      --no-f32-compare -o gpurun_out/r03_ids_c3_$i.json > gpurun_out/r03_ids_c3_$i.log 2>&1 || exit $?
  python3 -c "import json;d=json.load(open('gpurun_out/r03_ids_c3_$i.json'));print('c3', d['ms_per_step'], d['value'], d['roofline']['frac'], d['roofline']['dedup_prepass_ms_per_step'])"
done
