#!/bin/bash
# quick loop: kernel parity tests + in-batch microbench
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_kernels.py -q -m gpu -p no:cacheprovider -x > gpurun_out/tq.log 2>&1
rc=$?; tail -3 gpurun_out/tq.log; [ $rc -ne 0 ] && { grep -E "Error|assert" gpurun_out/tq.log | head -20; exit $rc; }
timeout -k 10 300 python tools/microbench_inbatch.py 65536 128 2>&1 | grep -v amdgpu.ids
timeout -k 10 300 python tools/microbench_inbatch.py 4096 128 2>&1 | grep -v amdgpu.ids
