#!/bin/bash
# round 4 (last): the whole GPU suite, smoke, the driver's default bench line and the same command
# under rocprofv3 --kernel-trace --stats
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread \
    > gpurun_out/r04_fin6_suite.log 2>&1
rc=$?; echo "suite rc=$rc"; tail -2 gpurun_out/r04_fin6_suite.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c 'import __graft_entry__ as g; g.smoke()' > gpurun_out/r04_fin6_smoke.log 2>&1 || exit $?
tail -1 gpurun_out/r04_fin6_smoke.log
timeout -k 10 900 python -u bench.py -o gpurun_out/r04_fin6_bench.json > gpurun_out/r04_fin6_bench.log 2>&1 || exit $?
python3 -c "import json; d=json.load(open('gpurun_out/r04_fin6_bench.json')); print(d['ms_per_step'], d['value'], d['roofline']['frac'], d['roofline']['achieved'])"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_fin6 -o p -- \
    python3 bench.py --extras off --steps 20 --warmup 3 -o gpurun_out/r04_fin6_bench_prof.json > gpurun_out/r04_fin6_prof.log 2>&1 || exit $?
f=$(find gpurun_out/prof_fin6 -name "*results.db" | head -1)
python3 tools/rocpd_stats.py $f gpurun_out/r04_c3_kernel_stats_fin6.csv 60 > gpurun_out/r04_c3_kernel_stats_fin6.txt 2>&1
rm -rf gpurun_out/prof_fin6
head -4 gpurun_out/r04_c3_kernel_stats_fin6.txt | cut -c1-150
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_fin6c2 -o c2 -- python3 bench.py --config c2 \
    --extras off --no-cpu-baseline --no-f32-compare --steps 20 --warmup 3 -o gpurun_out/r04_fin6_c2_prof.json \
    > gpurun_out/r04_fin6_c2_prof.log 2>&1 || exit $?
f=$(find gpurun_out/prof_fin6c2 -name "*results.db" | head -1)
python3 tools/rocpd_stats.py $f gpurun_out/r04_c2_kernel_stats_fin6.csv 60 > gpurun_out/r04_c2_kernel_stats_fin6.txt 2>&1
rm -rf gpurun_out/prof_fin6c2
timeout -k 10 300 python -u bench.py --config c2 --extras off --no-cpu-baseline --no-f32-compare --steps 100 \
    -o gpurun_out/r04_fin6_c2.json > gpurun_out/r04_fin6_c2.log 2>&1 || exit $?
python3 -c "import json; d=json.load(open('gpurun_out/r04_fin6_c2.json')); print('c2', d['ms_per_step'], d['value'])"
