#!/bin/bash
# round 2 probes: two-table gather variants, DCN-v2 planes vs staging stack, c2 and c5 bench lines
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/ab_gather_tables.py > gpurun_out/ab_gather_tables.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/microbench_dcn2_planes.py 16384 > gpurun_out/dcn2_planes_16k.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/microbench_dcn2_planes.py 65536 > gpurun_out/dcn2_planes_64k.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --config c2 --steps 50 --warmup 10 --cpu-seconds 3 -o gpurun_out/bench_c2.json > gpurun_out/bench_c2.log 2>&1 || exit $?
timeout -k 10 400 python bench.py --config c5 --steps 10 --warmup 3 --cpu-seconds 3 --no-f32-compare -o gpurun_out/bench_c5.json > gpurun_out/bench_c5.log 2>&1 || exit $?
head -80 gpurun_out/ab_gather_tables.log; cat gpurun_out/dcn2_planes_*.log
