#!/bin/bash
# round 3 (session 2): restored-tree check -- full GPU suite, default bench line
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/r03_t_suite.log 2>&1
rc=$?; echo "suite rc=$rc"; tail -3 gpurun_out/r03_t_suite.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 400 python -u bench.py -o gpurun_out/r03_t_bench.json > gpurun_out/r03_t_bench.log 2>&1 || exit $?
tail -c 600 gpurun_out/r03_t_bench.log
