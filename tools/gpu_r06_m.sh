#!/bin/bash
# Round 6: the row pass's P.K with K^T read ahead (IB_ROW_PREFETCH_A=1) — tests, A/B against the
# col-prefetch default — and the col prefetch A/B again in the other order (default first).
cd "$(dirname "$0")/.."
tag=${1:-r06m}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
RECSYS_HIP_LIB=_ablibs/ib_rpfa.so timeout -k 10 600 python -u -m pytest -x -v --timeout 400 --timeout-method thread \
    tests/test_gpu_inbatch_dedup.py > $out/tests_rpfa.log 2>&1
rc=$?; tail -n 2 $out/tests_rpfa.log; [ $rc -eq 0 ] || exit $rc
PROFAB_OUT=$out/ab_row bash tools/gpu_prof_ab.sh _ablibs/ib_cpf.so _ablibs/ib_rpfa.so || exit $?
PROFAB_OUT=$out/ab_col bash tools/gpu_prof_ab.sh _ablibs/ib_cpf.so _ablibs/ib_def.so
