#!/bin/bash
# Round 6: the dedup row pass with the S phase's next K rows read ahead (spf.so, IB_ROW_S_PREFETCH=1)
# against the release (rel.so), re-measured on the final tree: the pair digests of both builds
# (same products: bitwise), then the C3 kernel-statistics A/B in both orders, twice.
cd "$(dirname "$0")/.."
out=gpurun_out/${1:-r06ag}
mkdir -p $out
export TMPDIR=/tmp
for v in rel spf; do
  RECSYS_HIP_LIB=_ablibs/$v.so timeout -k 10 300 python3 -u tools/pair_digest.py > $out/digest_$v.txt 2>&1 || exit 1
done
diff $out/digest_rel.txt $out/digest_spf.txt && echo "digests equal"
PROFAB_OUT=$out/ab1 bash tools/gpu_prof_ab.sh _ablibs/rel.so _ablibs/spf.so | grep -E "row_m16|col_m16|total" || exit 1
PROFAB_OUT=$out/ab2 bash tools/gpu_prof_ab.sh _ablibs/spf.so _ablibs/rel.so | grep -E "row_m16|col_m16|total" || exit 1
PROFAB_OUT=$out/ab3 bash tools/gpu_prof_ab.sh _ablibs/rel.so _ablibs/spf.so | grep -E "row_m16|col_m16|total" || exit 1
PROFAB_OUT=$out/ab4 bash tools/gpu_prof_ab.sh _ablibs/spf.so _ablibs/rel.so | grep -E "row_m16|col_m16|total"
