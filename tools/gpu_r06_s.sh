#!/bin/bash
# Round 6: the row finalize with lane-parallel slot counts at 1 / 2 / 4 rows per wave, and the two
# pending read-ahead switches (IB_ROW_S_PREFETCH, WS_READ_AHEAD) against the release build:
# the release build's in-batch / gather tests, then C3 kernel-statistics A/Bs.
cd "$(dirname "$0")/.."
out=gpurun_out/${1:-r06s}
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
    tests/test_gpu_inbatch_dedup.py tests/test_gpu_c3_dedup_at_size.py tests/test_gpu_kernels.py -k "inbatch or gather or dedup or finalize or c3" \
    > $out/tests_release.log 2>&1
rc=$?; tail -n 2 $out/tests_release.log; [ $rc -eq 0 ] || exit $rc
PROFAB_OUT=$out/fin14 bash tools/gpu_prof_ab.sh _ablibs/fin1.so _ablibs/fin4.so || exit $?
PROFAB_OUT=$out/fin42 bash tools/gpu_prof_ab.sh _ablibs/fin4.so _ablibs/fin2.so || exit $?
PROFAB_OUT=$out/sp bash tools/gpu_prof_ab.sh _ablibs/fin4.so _ablibs/ab_sp.so || exit $?
PROFAB_OUT=$out/wsra bash tools/gpu_prof_ab.sh _ablibs/ab_wsra.so _ablibs/fin4.so
