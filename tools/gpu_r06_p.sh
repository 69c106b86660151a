#!/bin/bash
# Round 6: the weight-stationary GEMM with the next W fragment read ahead (WS_READ_AHEAD=1): the
# GEMM tests, then the C3 kernel-statistics A/B in both orders.
cd "$(dirname "$0")/.."
tag=${1:-r06p}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
RECSYS_HIP_LIB=_ablibs/ib_wsra.so timeout -k 10 600 python -u -m pytest -x -v --timeout 400 --timeout-method thread \
    tests/test_gpu_kernels.py tests/test_gpu_model.py -k "gemm or ws or tower or mlp or Dense or dense" > $out/tests_wsra.log 2>&1
rc=$?; tail -n 2 $out/tests_wsra.log; [ $rc -eq 0 ] || exit $rc
PROFAB_OUT=$out/ab1 bash tools/gpu_prof_ab.sh _ablibs/ib_r1.so _ablibs/ib_wsra.so || exit $?
PROFAB_OUT=$out/ab2 bash tools/gpu_prof_ab.sh _ablibs/ib_wsra.so _ablibs/ib_r1.so
