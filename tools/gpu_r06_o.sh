#!/bin/bash
# Round 6: the row pass's S phase with the next chunk's K rows read ahead (IB_ROW_S_PREFETCH=1):
# tests, then the C3 kernel-statistics A/B in both orders.
cd "$(dirname "$0")/.."
tag=${1:-r06o}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
RECSYS_HIP_LIB=_ablibs/ib_sp.so timeout -k 10 600 python -u -m pytest -x -v --timeout 400 --timeout-method thread \
    tests/test_gpu_inbatch_dedup.py > $out/tests_sp.log 2>&1
rc=$?; tail -n 2 $out/tests_sp.log; [ $rc -eq 0 ] || exit $rc
PROFAB_OUT=$out/ab1 bash tools/gpu_prof_ab.sh _ablibs/ib_r1.so _ablibs/ib_sp.so || exit $?
PROFAB_OUT=$out/ab2 bash tools/gpu_prof_ab.sh _ablibs/ib_sp.so _ablibs/ib_r1.so
