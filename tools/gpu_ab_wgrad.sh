#!/bin/bash
# dW kernel variants: parity tests on the default library, the tower-layer microbench per variant,
# then an alternating C3 A/B. Usage: tools/gpu_ab_wgrad.sh "libA libB ..." "libX libY ..."  (names in _ablibs/)
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -k "ws_wgrad or wgrad_bias or group_matches_single or mlp_wgrad" > gpurun_out/wg_tests.log 2>&1 || { tail -30 gpurun_out/wg_tests.log; exit 1; }
tail -1 gpurun_out/wg_tests.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_c3_dedup_at_size.py -x -q --timeout 200 --timeout-method thread -k distinct > gpurun_out/wg_distinct.log 2>&1 || { tail -30 gpurun_out/wg_distinct.log; exit 1; }
tail -1 gpurun_out/wg_distinct.log
for l in $1; do echo "== $l"; RECSYS_HIP_LIB=_ablibs/$l.so timeout -k 10 120 python tools/microbench_towers.py 65536 || exit 1; done
[ -n "$2" ] && bash tools/gpu_ab_c3.sh $(for l in $2; do echo _ablibs/$l.so; done)
exit 0
