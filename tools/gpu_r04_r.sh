#!/bin/bash
# round 4: the backward reusing its forward's workspace (RS_INBATCH_FWD_WS): in-batch tests, then
# c3 / c2 lines
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests/test_gpu_inbatch_dedup.py tests/test_gpu_kernels.py tests/test_gpu_model.py \
    tests/test_gpu_c3_dedup_at_size.py tests/test_gpu_production_sizes.py -m gpu -x -q --timeout 300 \
    --timeout-method thread > gpurun_out/r04_r_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r04_r_tests.log; [ $rc -eq 0 ] || exit $rc
for c in c3 c2 c3 c2; do
  timeout -k 10 300 python -u bench.py --config $c --extras off --no-cpu-baseline --no-f32-compare --steps 40 \
      -o gpurun_out/r04_r_$c.json > gpurun_out/r04_r_$c.log 2>&1 || exit $?
  python3 -c "import json; d=json.load(open('gpurun_out/r04_r_$c.json')); print('$c', d['ms_per_step'], d['value'], d['roofline']['frac'])"
done
# the driver's N > 1 command, rehearsed with 2 ranks on this one GPU over gloo (RCCL refuses two
# ranks on one device): the eager default (deduplicating exchange) and --graph (padded exchange)
for extra in "" "--graph"; do
  RS_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
      --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 4 --warmup 2 --extras off \
      --no-cpu-baseline --no-f32-compare $extra > gpurun_out/r04_r_dp2$extra.log 2>&1 || { tail -20 gpurun_out/r04_r_dp2$extra.log; exit 1; }
  tail -1 gpurun_out/r04_r_dp2$extra.log | cut -c1-300
done
