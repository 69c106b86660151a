#!/bin/bash
# round 4 closing: the driver's N > 1 command rehearsed with 2 ranks on one GPU over gloo (eager
# default and --graph)
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
for extra in "" "--graph"; do
  RS_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
      --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 4 --warmup 2 --extras off \
      --no-cpu-baseline --no-f32-compare $extra > gpurun_out/r04_dp2_close$extra.log 2>&1 || { tail -20 gpurun_out/r04_dp2_close$extra.log; exit 1; }
  tail -1 gpurun_out/r04_dp2_close$extra.log | cut -c1-200
done
