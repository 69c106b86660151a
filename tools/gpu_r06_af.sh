#!/bin/bash
# Round 6: the masked dX of the weight-stationary GEMM at K = 128 on 128-column slices
# (mk128.so, WS_MASKED_K128_NW=128: the mask in 64 VGPRs, half the slices) vs the release 64-column
# slices (rel.so): the ws GEMM / tower tests on mk128, a bitwise digest of the pair outputs is not
# needed (the slice width does not change any sum), then the C3 kernel statistics in both orders.
cd "$(dirname "$0")/.."
out=gpurun_out/${1:-r06af}
mkdir -p $out
export TMPDIR=/tmp
RECSYS_HIP_LIB=_ablibs/mk128.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
    tests/test_gpu_kernels.py -k "ws_gemm or wgrad or towers" > $out/tests_mk128.log 2>&1
rc=$?; tail -n 1 $out/tests_mk128.log; [ $rc -eq 0 ] || exit $rc
PROFAB_OUT=$out/ab1 bash tools/gpu_prof_ab.sh _ablibs/rel.so _ablibs/mk128.so | grep -E "gemm_ws|total" || exit 1
PROFAB_OUT=$out/ab2 bash tools/gpu_prof_ab.sh _ablibs/mk128.so _ablibs/rel.so | grep -E "gemm_ws|total"
