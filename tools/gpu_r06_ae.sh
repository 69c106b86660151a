#!/bin/bash
# Round 6: the large-batch dW's K-slice count against its slab reduction: release (rel.so, ~256
# workgroups per problem, >= 512 rows per slice) vs variants V1 V2 (default: half the slices,
# wgs128.so, WGWS_WGS=128; >= 1024 rows per slice, mink1k.so, WGWS_MINK=1024): the dW tests on each
# variant, then C3 kernel statistics (rel vs V1 in both orders, rel vs V2).
# Usage: tools/gpu_r06_ae.sh TAG [V1 V2]
cd "$(dirname "$0")/.."
out=gpurun_out/${1:-r06ae}
mkdir -p $out
export TMPDIR=/tmp
v1=${2:-wgs128}; v2=${3:-mink1k}
for v in $v1 $v2; do
  RECSYS_HIP_LIB=_ablibs/$v.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
      tests/test_gpu_kernels.py -k "wgrad or towers" > $out/tests_$v.log 2>&1
  rc=$?; tail -n 1 $out/tests_$v.log; [ $rc -eq 0 ] || exit $rc
done
PROFAB_OUT=$out/ab1 bash tools/gpu_prof_ab.sh _ablibs/rel.so _ablibs/$v1.so | grep -E "wgrad|slab|total" || exit 1
PROFAB_OUT=$out/ab2 bash tools/gpu_prof_ab.sh _ablibs/$v1.so _ablibs/rel.so | grep -E "wgrad|slab|total" || exit 1
PROFAB_OUT=$out/ab3 bash tools/gpu_prof_ab.sh _ablibs/rel.so _ablibs/$v2.so | grep -E "wgrad|slab|total"
