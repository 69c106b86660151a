#!/bin/bash
# Round 6: the deduplicated row pass per owned subtile (IB_ROW_SPLIT_UB=1, su1.so = release) against
# the phase form (su0.so): the in-batch tests on su1, a bitwise cross-check of the two builds'
# pair outputs at the C3 shape, then the C3 kernel-statistics A/B in both orders.
cd "$(dirname "$0")/.."
out=gpurun_out/${1:-r06aa}
mkdir -p $out
export TMPDIR=/tmp
RECSYS_HIP_LIB=_ablibs/su1.so timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
    tests/test_gpu_inbatch_dedup.py tests/test_gpu_c3_dedup_at_size.py > $out/tests_su1.log 2>&1
rc=$?; tail -n 1 $out/tests_su1.log; [ $rc -eq 0 ] || exit $rc
for v in su0 su1; do
  RECSYS_HIP_LIB=_ablibs/$v.so timeout -k 10 300 python3 -u tools/pair_digest.py > $out/digest_$v.txt 2>&1 || exit 1
done
diff $out/digest_su0.txt $out/digest_su1.txt && echo "digests equal"
PROFAB_OUT=$out/ab1 bash tools/gpu_prof_ab.sh _ablibs/su0.so _ablibs/su1.so | grep -E "row_m16|col_m16|total" || exit 1
PROFAB_OUT=$out/ab2 bash tools/gpu_prof_ab.sh _ablibs/su1.so _ablibs/su0.so | grep -E "row_m16|col_m16|total"
