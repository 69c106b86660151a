#!/bin/bash
# round 4: the driver's default bench line, then the same command under rocprofv3 --kernel-trace --stats
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u bench.py -o gpurun_out/r04_final_bench.json > gpurun_out/r04_final_bench.log 2>&1 || exit $?
python3 -c "import json; d=json.load(open('gpurun_out/r04_final_bench.json')); print(d['ms_per_step'], d['value'], d['roofline']['frac'])"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r04final -o p -- \
    python3 bench.py --extras off --steps 20 --warmup 3 -o gpurun_out/r04_final_bench_prof.json > gpurun_out/r04_final_prof.log 2>&1 || exit $?
f=$(find gpurun_out/prof_r04final -name "*results.db" | head -1)
python3 tools/rocpd_stats.py $f gpurun_out/r04_c3_kernel_stats_final.csv 60 > gpurun_out/r04_c3_kernel_stats_final.txt 2>&1
rm -rf gpurun_out/prof_r04final
head -6 gpurun_out/r04_c3_kernel_stats_final.txt | cut -c1-150
