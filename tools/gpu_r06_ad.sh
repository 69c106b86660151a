#!/bin/bash
# Round 6: the split kernels at 4 waves per workgroup, two workgroups per CU (IBX_NW=4, nw4.so;
# 128-row stream-K blocks, 512 workgroups) against the release 8-wave form (nw8.so): the in-batch
# tests on nw4, the two builds' pair digests (not bitwise: the partial-slot merge order changes),
# then the C3 kernel-statistics A/B in both orders.
cd "$(dirname "$0")/.."
out=gpurun_out/${1:-r06ad}
mkdir -p $out
export TMPDIR=/tmp
RECSYS_HIP_LIB=_ablibs/nw4.so timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
    tests/test_gpu_inbatch_dedup.py tests/test_gpu_c3_dedup_at_size.py > $out/tests_nw4.log 2>&1
rc=$?; tail -n 1 $out/tests_nw4.log; [ $rc -eq 0 ] || exit $rc
for v in nw8 nw4; do
  RECSYS_HIP_LIB=_ablibs/$v.so timeout -k 10 300 python3 -u tools/pair_digest.py > $out/digest_$v.txt 2>&1 || exit 1
done
diff $out/digest_nw8.txt $out/digest_nw4.txt && echo "digests equal"
PROFAB_OUT=$out/ab1 bash tools/gpu_prof_ab.sh _ablibs/nw8.so _ablibs/nw4.so | grep -E "row_m16|col_m16|finalize|total" || exit 1
PROFAB_OUT=$out/ab2 bash tools/gpu_prof_ab.sh _ablibs/nw4.so _ablibs/nw8.so | grep -E "row_m16|col_m16|finalize|total"
