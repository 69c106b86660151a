#!/bin/bash
# round 3: multi-rank GPU tests, the default bench line with its c5/c4 sub-records, a 2-rank gloo
# rehearsal of bench.py, and the same-GPU RCCL probe
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_multirank.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r03_multirank.log 2>&1
rc=$?
echo "multirank rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 -o gpurun_out/r03_bench1.json > gpurun_out/r03_bench1.log 2>&1 || exit $?
echo "bench ok"
RS_DIST_BACKEND=gloo timeout -k 10 300 python -u bench.py --gpus 2 --steps 5 --warmup 2 --no-cpu-baseline --no-f32-compare -o gpurun_out/r03_bench_2rank_gloo.json > gpurun_out/r03_bench_2rank_gloo.log 2>&1 || exit $?
echo "2-rank ok"
timeout -k 10 90 python -m torch.distributed.run --nnodes=1 --nproc-per-node=2 --master-addr 127.0.0.1 --master-port 29533 tools/r03_nccl_same_gpu.py > gpurun_out/r03_nccl_same_gpu.log 2>&1
echo "nccl probe rc=$?"
exit 0
