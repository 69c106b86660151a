#!/bin/bash
# round 2: full GPU test suite (incl. the production-size parity tests), then the c3 bench line
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread \
  --durations=15 > gpurun_out/tests.log 2>&1
rc=$?; tail -25 gpurun_out/tests.log
if [ $rc -ne 0 ]; then grep -E "^E |FAILED|Error" gpurun_out/tests.log | head -40; exit $rc; fi
timeout -k 10 600 python bench.py --steps 10 --warmup 3 -o gpurun_out/bench_c3.json > gpurun_out/bench_c3.log 2>&1
rc=$?; tail -c 4000 gpurun_out/bench_c3.log; exit $rc
