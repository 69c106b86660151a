#!/bin/bash
# Round 6: col pass timing probes against the release build: probe2 = P formed in the first step of
# a segment only and reused (realistic values, wrong results); fresh0 = MFMAs accumulate into the
# running O' (no fresh-tile adds; the round-4 numerics).
cd "$(dirname "$0")/.."
out=gpurun_out/${1:-r06v}
mkdir -p $out
export TMPDIR=/tmp
for v in probe2 fresh0; do
  PROFAB_OUT=$out/$v bash tools/gpu_prof_ab.sh _ablibs/chain1.so _ablibs/$v.so 2>&1 | grep -E "col_m16|row_m16|total" || exit 1
done
