#!/bin/bash
# round 2: c3 kernel stats after the col-pass DMA change; the c5 cross stack at B = 16384 and 65536
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c3b -o c3 -- \
    python3 bench.py --config c3 --steps 10 --warmup 2 --no-cpu-baseline --no-f32-compare -o gpurun_out/prof_bench_c3b.json > gpurun_out/prof_c3b.log 2>&1 || { tail -20 gpurun_out/prof_c3b.log; exit 1; }
f=$(find gpurun_out/prof_c3b -name '*kernel_stats.csv' | head -1); python tools/kstats.py $f 6
timeout -k 10 300 python -u tools/microbench_dcn2_planes.py 16384 > gpurun_out/dcn2_planes_16k.log 2>&1 || exit $?
timeout -k 10 400 python -u tools/microbench_dcn2_planes.py 65536 > gpurun_out/dcn2_planes_64k.log 2>&1 || exit $?
cat gpurun_out/dcn2_planes_16k.log gpurun_out/dcn2_planes_64k.log
