#!/bin/bash
# Round 6: the col pass's per-accumulator product chains (IB_COL_CHAIN=1, release: the fresh-tile
# adds six MFMAs after their chain, P slices spread over the d-tiles) against the interleaved form
# (chain0.so): the in-batch tests and the GEMM tests on the release build, then the C3 A/B both orders.
cd "$(dirname "$0")/.."
out=gpurun_out/${1:-r06t}
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
    tests/test_gpu_inbatch_dedup.py tests/test_gpu_c3_dedup_at_size.py tests/test_gpu_kernels.py \
    > $out/tests_release.log 2>&1
rc=$?; tail -n 2 $out/tests_release.log; [ $rc -eq 0 ] || exit $rc
PROFAB_OUT=$out/ab1 bash tools/gpu_prof_ab.sh _ablibs/chain0.so _ablibs/chain1.so || exit $?
PROFAB_OUT=$out/ab2 bash tools/gpu_prof_ab.sh _ablibs/chain1.so _ablibs/chain0.so
