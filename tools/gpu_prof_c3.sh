#!/bin/bash
# rocprofv3 kernel stats of the c3 bench (eager, no f32 comparison, no CPU baseline)
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c3 -o c3 -- \
    python3 bench.py --config ${CFG:-c3} --steps 10 --warmup 2 --no-cpu-baseline --no-f32-compare -o gpurun_out/prof_bench_c3.json > gpurun_out/prof_c3.log 2>&1 || { tail -20 gpurun_out/prof_c3.log; exit 1; }
f=$(find gpurun_out/prof_c3 -name '*kernel_stats.csv' | head -1); python tools/kstats.py $f 45
