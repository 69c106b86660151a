#!/bin/bash
# round 3 (session 2): full GPU suite, then the default bench line and its rocprofv3 kernel stats
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/r03_final_suite.log 2>&1
rc=$?; echo "suite rc=$rc"; tail -3 gpurun_out/r03_final_suite.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 400 python -u bench.py -o gpurun_out/r03_final_bench.json > gpurun_out/r03_final_bench.log 2>&1 || exit $?
tail -c 300 gpurun_out/r03_final_bench.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_final -o z -- \
    python3 bench.py --no-cpu-baseline -o gpurun_out/r03_final_bench_prof.json > gpurun_out/r03_final_prof.log 2>&1 || exit $?
f=$(find gpurun_out/prof_final -name '*kernel_stats.csv' | head -1); python3 tools/kstats.py $f 30 > gpurun_out/r03_final_kstats.txt
head -12 gpurun_out/r03_final_kstats.txt
