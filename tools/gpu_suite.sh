#!/bin/bash
# The whole -m gpu suite, then smoke(): tools/gpu_suite.sh TAG [pytest args...]
# (logs: gpurun_out/TAG_suite.log, gpurun_out/TAG_smoke.log)
cd "$(dirname "$0")/.."
tag=${1:-run}; shift
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -x "$@" \
    > gpurun_out/${tag}_suite.log 2>&1
rc=$?; echo "suite rc=$rc"; tail -5 gpurun_out/${tag}_suite.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c 'import __graft_entry__ as g; g.smoke()' > gpurun_out/${tag}_smoke.log 2>&1 || exit $?
tail -1 gpurun_out/${tag}_smoke.log
