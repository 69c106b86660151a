#!/bin/bash
# Round 6: saddr LDS-DMA addressing (default build) and the staggered row pass with the late waves'
# copy at the block start: tests, then C3 kernel-statistics A/B runs against the previous build.
cd "$(dirname "$0")/.."
tag=${1:-r06j}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 400 --timeout-method thread \
    tests/test_gpu_inbatch_dedup.py > $out/tests.log 2>&1
rc=$?; tail -n 2 $out/tests.log; [ $rc -eq 0 ] || exit $rc
RECSYS_HIP_LIB=_ablibs/ib_stg3.so timeout -k 10 600 python -u -m pytest -x -v --timeout 400 --timeout-method thread \
    tests/test_gpu_inbatch_dedup.py > $out/tests_stg3.log 2>&1
rc=$?; tail -n 2 $out/tests_stg3.log; [ $rc -eq 0 ] || exit $rc
PROFAB_OUT=$out/ab_saddr bash tools/gpu_prof_ab.sh _ablibs/ib_base.so _ablibs/ib_saddr.so || exit $?
PROFAB_OUT=$out/ab_stg3 bash tools/gpu_prof_ab.sh _ablibs/ib_saddr.so _ablibs/ib_stg3.so
bash tools/gpu_pmc_dedup.sh r06 > gpurun_out/$tag/pmc_dedup.log 2>&1; tail -n 3 gpurun_out/$tag/pmc_dedup.log
