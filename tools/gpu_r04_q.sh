#!/bin/bash
# round 4: the staggered-halves row pass (RS_IB_ROW_PIPE=1) — dedup tests under it, then c3 A/B
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
RS_IB_ROW_PIPE=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_inbatch_dedup.py tests/test_gpu_c3_dedup_at_size.py \
    -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r04_q_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/r04_q_tests.log; [ $rc -eq 0 ] || exit $rc
for v in 0 1 0 1; do
  RS_IB_ROW_PIPE=$v timeout -k 10 300 python -u bench.py --extras off --no-cpu-baseline --no-f32-compare --steps 30 \
      -o gpurun_out/r04_q_$v.json > /dev/null 2>&1 || exit $?
  python3 -c "import json; d=json.load(open('gpurun_out/r04_q_$v.json')); print('pipe $v', d['ms_per_step'], d['roofline']['frac'], d['roofline']['avg_launch_ms'])"
done
