#!/bin/bash
# round 3: the c3 line with the deduplicated pair (bench's per-call FLOPs) and its kernel statistics
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u bench.py --config c3 --steps 30 --warmup 5 --no-cpu-baseline --extras off \
    -o gpurun_out/r03_c3_dedup2.json > gpurun_out/r03_c3_dedup2.log 2>&1 || exit $?
echo "c3 ok"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r03_c3dd -o run -- \
    python3 bench.py --config c3 --steps 20 --warmup 3 --no-cpu-baseline --no-f32-compare --extras off \
    -o gpurun_out/prof_r03_c3dd.json > gpurun_out/prof_r03_c3dd.log 2>&1 || exit $?
echo "prof ok"
