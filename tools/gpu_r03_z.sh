#!/bin/bash
# round 3 (session 2): full GPU suite, PMC traffic of the c4 call on the bound-first path, then the
# default bench line and its rocprofv3 kernel stats
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/r03_z_suite.log 2>&1
rc=$?; echo "suite rc=$rc"; tail -3 gpurun_out/r03_z_suite.log
if [ $rc -ne 0 ]; then exit $rc; fi
d=gpurun_out/pmc_c4b
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 150 rocprofv3 --kernel-trace --pmc $c --output-format csv -d $d/$c -o x -- \
      python3 tools/traffic_probe.py c4 4 > $d.$c.log 2>&1 || { echo "pmc $c failed"; exit 1; }
done
python3 tools/traffic_summary.py gpurun_out/r03_pmc_c4_boundfirst.json c4=$d:4
timeout -k 10 400 python -u bench.py -o gpurun_out/r03_z_bench.json > gpurun_out/r03_z_bench.log 2>&1 || exit $?
tail -c 300 gpurun_out/r03_z_bench.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_z -o z -- \
    python3 bench.py --no-cpu-baseline -o gpurun_out/r03_z_bench_prof.json > gpurun_out/r03_z_prof.log 2>&1 || exit $?
f=$(find gpurun_out/prof_z -name '*kernel_stats.csv' | head -1); python3 tools/kstats.py $f 30 > gpurun_out/r03_z_kstats.txt
head -12 gpurun_out/r03_z_kstats.txt
