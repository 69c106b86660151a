#!/bin/bash
# round 2 quick check: one test file pattern (arg 1) then a c3 bench line (arg 2 = extra bench args)
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu -k "${1:-gather}" -p no:cacheprovider --timeout 300 --timeout-method thread \
  > gpurun_out/tests_quick.log 2>&1
rc=$?; tail -5 gpurun_out/tests_quick.log
if [ $rc -ne 0 ]; then grep -E "^E |FAILED|Error" gpurun_out/tests_quick.log | head -40; exit $rc; fi
timeout -k 10 600 python bench.py --steps 10 --warmup 3 --no-f32-compare --cpu-seconds 2 $2 -o gpurun_out/bench_quick.json > gpurun_out/bench_quick.log 2>&1
rc=$?; tail -c 3000 gpurun_out/bench_quick.log; exit $rc
