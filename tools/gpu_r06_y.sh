#!/bin/bash
# Round 6: the id plan's merge-sort block size (RS_PLAN_SORT_BS x RS_PLAN_SORT_IPT = 4096 / 8192
# items per sorted block instead of rocprim's 1024): the plan / dedup tests on each variant, then
# the C3 kernel-statistics A/Bs against the release build.
cd "$(dirname "$0")/.."
out=gpurun_out/${1:-r06y}
mkdir -p $out
export TMPDIR=/tmp
for v in sort4k sort8k; do
  RECSYS_HIP_LIB=_ablibs/$v.so timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
      tests/test_gpu_inbatch_dedup.py tests/test_gpu_dp_sparse.py > $out/tests_$v.log 2>&1
  rc=$?; echo "$v tests rc=$rc"; tail -n 1 $out/tests_$v.log; [ $rc -eq 0 ] || exit $rc
done
PROFAB_OUT=$out/s4 bash tools/gpu_prof_ab.sh _ablibs/sort0.so _ablibs/sort4k.so | grep -E "trampoline|lookback|total" || exit 1
PROFAB_OUT=$out/s8 bash tools/gpu_prof_ab.sh _ablibs/sort0.so _ablibs/sort8k.so | grep -E "trampoline|lookback|total"
