#!/bin/bash
# round 4: the full GPU suite after the caller-owned reduction queue (ABI 2), then smoke()
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/r04_b_suite.log 2>&1
rc=$?; echo "suite rc=$rc"; tail -15 gpurun_out/r04_b_suite.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -c 'import __graft_entry__ as g; g.smoke()' > gpurun_out/r04_b_smoke.log 2>&1 || exit $?
tail -2 gpurun_out/r04_b_smoke.log
