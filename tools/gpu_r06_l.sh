#!/bin/bash
# Round 6: the col pass with the next d-tile's U^T operand read ahead (IB_COL_PREFETCH_A=1): its
# in-batch tests, then the C3 kernel-statistics A/B against the default build.
cd "$(dirname "$0")/.."
tag=${1:-r06l}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
RECSYS_HIP_LIB=_ablibs/ib_pfa.so timeout -k 10 600 python -u -m pytest -x -v --timeout 400 --timeout-method thread \
    tests/test_gpu_inbatch_dedup.py > $out/tests_pfa.log 2>&1
rc=$?; tail -n 2 $out/tests_pfa.log; [ $rc -eq 0 ] || exit $rc
PROFAB_OUT=$out/ab bash tools/gpu_prof_ab.sh _ablibs/ib_def.so _ablibs/ib_pfa.so
