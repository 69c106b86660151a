#!/bin/bash
# round 3: the whole GPU suite, smoke(), and the driver's default bench line (c3 + extras)
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/r03_gpu_suite_run2.log 2>&1
rc=$?; echo "suite rc=$rc"
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r03_smoke2.log 2>&1 || exit $?
timeout -k 10 900 python -u bench.py -o gpurun_out/r03_bench_default2.json > gpurun_out/r03_bench_default2.log 2>&1 || exit $?
echo "bench ok"
