#!/bin/bash
# round 3 (session 2): kernel trace of the two-phase top-k (Q = 1024, 12.5M x 128, Gaussian) and
# the deduplicated in-batch pair's PMC passes
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
GAUSS=1 PREC=6 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_tp -o tp -- \
    python3 tools/microbench_topk.py 12500000 100 1024 > gpurun_out/r03_w_tp.log 2>&1 || exit $?
f=$(find gpurun_out/prof_tp -name '*kernel_stats.csv' | head -1); python3 tools/kstats.py $f 12
bash tools/gpu_r03_pmc_dedup.sh
