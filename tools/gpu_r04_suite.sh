#!/bin/bash
# round 4: the whole GPU suite, smoke, and the deduplicated pair's PMC passes
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread \
    > gpurun_out/r04_suite.log 2>&1
rc=$?; echo "suite rc=$rc"; tail -3 gpurun_out/r04_suite.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c 'import __graft_entry__ as g; g.smoke()' > gpurun_out/r04_smoke.log 2>&1 || exit $?
tail -1 gpurun_out/r04_smoke.log
bash tools/gpu_r04_pmc_dedup.sh > gpurun_out/r04_pmc_run.log 2>&1 || { tail -5 gpurun_out/r04_pmc_run.log; exit 1; }
tail -25 gpurun_out/r04_pmc_ibdedup.txt | cut -c1-140
