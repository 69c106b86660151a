#!/bin/bash
# Round 6: col pass timing probes against the release build (wrong results, timing only):
# probe1 = no exponentials in P, probe2 = no P formed at all, probe3 = no fresh-tile adds.
cd "$(dirname "$0")/.."
out=gpurun_out/${1:-r06u}
mkdir -p $out
export TMPDIR=/tmp
for i in 1 2 3; do
  PROFAB_OUT=$out/p$i bash tools/gpu_prof_ab.sh _ablibs/chain1.so _ablibs/probe$i.so 2>&1 | grep -E "col_m16|row_m16|total" || exit 1
done
