#!/bin/bash
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c4 -o c4 -- \
    python3 bench.py --config c4 --steps 5 --warmup 2 --no-cpu-baseline --no-f32-compare -o gpurun_out/prof_bench_c4.json > gpurun_out/prof_c4.log 2>&1
echo "rc=$?"
