#!/bin/bash
# Round 6: rows per wave of the distinct-id lookup (GATHER_IDS_RPW 64 / 32 / 16), A B A order.
cd "$(dirname "$0")/.."
out=gpurun_out/${1:-r06q}
mkdir -p $out
for v in g64 g16 g32 g64 g16; do
  RECSYS_HIP_LIB=_ablibs/$v.so timeout -k 10 240 python3 -u tools/microbench_gather_ids.py >> $out/gather_ids.log 2>&1 || exit $?
done
cat $out/gather_ids.log
