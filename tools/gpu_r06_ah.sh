#!/bin/bash
# Round 6: the row finalize with 6 / 8 O partials per row loaded up front (pre6.so / pre8.so,
# IB_FIN_PRE) against the release 4 (rel.so): pair digests (same sums: bitwise), then C3 kernel
# statistics, rel vs V1 in both orders and rel vs V2. Usage: tools/gpu_r06_ah.sh TAG [V1 V2]
cd "$(dirname "$0")/.."
out=gpurun_out/${1:-r06ah}
mkdir -p $out
export TMPDIR=/tmp
v1=${2:-pre6}; v2=${3:-pre8}
for v in rel $v1 $v2; do
  RECSYS_HIP_LIB=_ablibs/$v.so timeout -k 10 300 python3 -u tools/pair_digest.py > $out/digest_$v.txt 2>&1 || exit 1
done
diff $out/digest_rel.txt $out/digest_$v1.txt && diff $out/digest_rel.txt $out/digest_$v2.txt && echo "digests equal"
PROFAB_OUT=$out/ab1 bash tools/gpu_prof_ab.sh _ablibs/rel.so _ablibs/$v1.so | grep -E "finalize|total" || exit 1
PROFAB_OUT=$out/ab2 bash tools/gpu_prof_ab.sh _ablibs/$v1.so _ablibs/rel.so | grep -E "finalize|total" || exit 1
PROFAB_OUT=$out/ab3 bash tools/gpu_prof_ab.sh _ablibs/rel.so _ablibs/$v2.so | grep -E "finalize|total"
