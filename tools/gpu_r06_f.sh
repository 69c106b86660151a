#!/bin/bash
# Round 6: the DP rehearsals (gpu_r06_e.sh), then the col pass's transposed user image A/B
# (IB_COL_TIMG=0 vs 1, C3 bench kernel statistics).
cd "$(dirname "$0")/.."
tag=${1:-r06f}
bash tools/gpu_r06_e.sh $tag || exit $?
PROFAB_OUT=gpurun_out/$tag/ab bash tools/gpu_prof_ab.sh _ablibs/ib_timg0.so _ablibs/ib_timg1.so
PROFAB_OUT=gpurun_out/$tag/ab2 bash tools/gpu_prof_ab.sh _ablibs/ib_timg1.so _ablibs/ib_prio1.so
