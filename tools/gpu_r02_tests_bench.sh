#!/bin/bash
# selected GPU parity tests (KSEL) then bench lines (CONFIGS) for a quick check of one change
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu -k "${KSEL:-sparse or dedupe or multi_table or distributed or inbatch or model or dcn2}" \
    -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/sm_tests.log 2>&1; rc=$?
tail -3 gpurun_out/sm_tests.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/sm_tests.log | head -20; exit $rc; }
for c in ${CONFIGS:-c5 c2 c3}; do
  timeout -k 10 300 python bench.py --config $c --steps 20 --warmup 3 --no-cpu-baseline --no-f32-compare -o gpurun_out/sm_$c.json > gpurun_out/sm_$c.log 2>&1 || { tail -5 gpurun_out/sm_$c.log; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/sm_$c.json'));print('$c', d['value'], d['unit'], d['ms_per_step'])"
done
