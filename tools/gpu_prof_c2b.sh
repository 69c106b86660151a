#!/bin/bash
# rocprofv3 kernel stats of the c2 bench (hipGraph replay): per-step launch list
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c2 -o c2 -- \
    python3 bench.py --config c2 --steps 50 --warmup 5 --no-cpu-baseline --no-f32-compare -o gpurun_out/prof_bench_c2.json > gpurun_out/prof_c2.log 2>&1 || { tail -20 gpurun_out/prof_c2.log; exit 1; }
f=$(find gpurun_out/prof_c2 -name '*kernel_stats.csv' | head -1); python tools/kstats.py $f 60 > gpurun_out/c2_kstats.txt; cat gpurun_out/c2_kstats.txt
