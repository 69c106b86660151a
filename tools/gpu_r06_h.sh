#!/bin/bash
# Round 6: the staggered row pass without in-loop spills (IB_ROW_STAGGER=1 build): its tests, then
# the C3 kernel-statistics A/B against the default build.
cd "$(dirname "$0")/.."
tag=${1:-r06h}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
RECSYS_HIP_LIB=_ablibs/ib_stg1c.so timeout -k 10 600 python -u -m pytest -x -v --timeout 400 --timeout-method thread \
    tests/test_gpu_inbatch_dedup.py > $out/tests_stg1c.log 2>&1
rc=$?; tail -n 2 $out/tests_stg1c.log; [ $rc -eq 0 ] || exit $rc
PROFAB_OUT=$out/ab_stg bash tools/gpu_prof_ab.sh _ablibs/ib_base.so _ablibs/ib_stg1c.so
