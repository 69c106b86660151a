#!/bin/bash
# In-batch pass variants: the dedup / pair parity tests on the default library, then an alternating
# C3 A/B (step + per-entry pair times). Usage: tools/gpu_ab_ib.sh libA.so libB.so ...
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_inbatch_dedup.py tests/test_gpu_c3_dedup_at_size.py -x -q --timeout 300 --timeout-method thread > gpurun_out/ib_tests.log 2>&1 || { tail -30 gpurun_out/ib_tests.log; exit 1; }
tail -1 gpurun_out/ib_tests.log
bash tools/gpu_ab_c3.sh "$@"
