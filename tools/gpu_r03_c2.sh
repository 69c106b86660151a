#!/bin/bash
# round 3 (session 2): c2 graphed step kernel trace (launches per step and their times)
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c2 -o c2 -- \
    python3 bench.py --config c2 --steps 100 --warmup 10 --no-cpu-baseline --extras off --no-f32-compare \
    -o gpurun_out/r03_c2_prof_line.json > gpurun_out/r03_c2_prof.log 2>&1 || exit $?
f=$(find gpurun_out/prof_c2 -name '*kernel_stats.csv' | head -1); python3 tools/kstats.py $f 60 > gpurun_out/r03_c2_kstats.txt
timeout -k 10 300 python3 bench.py --config c2 --steps 300 --warmup 20 --no-cpu-baseline --extras off --no-f32-compare \
    -o gpurun_out/r03_c2_line.json > gpurun_out/r03_c2_line.log 2>&1 || exit $?
python3 -c "import json;d=json.load(open('gpurun_out/r03_c2_line.json'));print('c2', d['ms_per_step'], d['value'])"
