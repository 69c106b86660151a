#!/bin/bash
# round 3: the captured data-parallel step (RCCL, one rank), then the c2 line and its kernel stats
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_multirank.py -v -s --timeout 240 --timeout-method thread \
    -k graphed > gpurun_out/r03_graph_dp.log 2>&1
rc=$?; echo "graph dp rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py --config c2 --steps 100 --warmup 5 --no-cpu-baseline -o gpurun_out/r03_c2.json \
    > gpurun_out/r03_c2.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r03_c2 -o run -- \
    python3 bench.py --config c2 --steps 50 --warmup 2 --no-cpu-baseline --no-f32-compare \
    -o gpurun_out/prof_r03_c2.json > gpurun_out/prof_r03_c2.log 2>&1 || exit $?
echo "c2 ok"
