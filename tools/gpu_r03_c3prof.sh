#!/bin/bash
# round 3 (session 2): c3 kernel trace at the final kernels (50 timed steps, extras off)
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c3 -o c3 -- \
    python3 bench.py --config c3 --steps 50 --warmup 3 --no-cpu-baseline --extras off --no-f32-compare \
    -o gpurun_out/r03_c3_prof_line.json > gpurun_out/r03_c3_prof.log 2>&1 || exit $?
f=$(find gpurun_out/prof_c3 -name '*kernel_stats.csv' | head -1); python3 tools/kstats.py $f 60 > gpurun_out/r03_c3_kstats.txt
head -5 gpurun_out/r03_c3_kstats.txt
