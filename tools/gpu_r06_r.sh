#!/bin/bash
# Round 6: the row finalize at 4 rows per wave (IB_FIN_RPW=4, release) against one row per wave
# (fin1.so): the in-batch tests on the release build, then the C3 kernel-statistics A/B both orders.
cd "$(dirname "$0")/.."
out=gpurun_out/${1:-r06r}
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
    tests/test_gpu_inbatch_dedup.py tests/test_gpu_c3_dedup_at_size.py > $out/tests_fin4.log 2>&1
rc=$?; tail -n 2 $out/tests_fin4.log; [ $rc -eq 0 ] || exit $rc
PROFAB_OUT=$out/ab1 bash tools/gpu_prof_ab.sh _ablibs/fin1.so _ablibs/fin4.so || exit $?
PROFAB_OUT=$out/ab2 bash tools/gpu_prof_ab.sh _ablibs/fin4.so _ablibs/fin8.so
