#!/bin/bash
# round 2: in-batch tests (incl. the B = 65536 production-size test), then the c3 and c2 bench lines
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu -k "inbatch or c3 or graph or model" -p no:cacheprovider \
  --timeout 300 --timeout-method thread > gpurun_out/tests_ib.log 2>&1
rc=$?; tail -3 gpurun_out/tests_ib.log
if [ $rc -ne 0 ]; then grep -E "^E |FAILED|Error" gpurun_out/tests_ib.log | head -40; exit $rc; fi
for c in c3 c2; do
  timeout -k 10 400 python bench.py --config $c --steps 20 --warmup 5 --no-cpu-baseline --no-f32-compare -o gpurun_out/bench_$c.json > gpurun_out/bench_$c.log 2>&1 || { tail -20 gpurun_out/bench_$c.log; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/bench_$c.json')); r=d['roofline']; print('$c', d['ms_per_step'], d['value'], r['frac'], r['avg_launch_ms'])"
done
