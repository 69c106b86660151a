#!/bin/bash
# round 3: top-k experiments + towers baseline (gpu_r03_c.sh), then the multi-rank tests and the
# bench lines (gpu_r03_b.sh)
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
bash tools/gpu_r03_c.sh > gpurun_out/r03_c.log 2>&1 || { echo "c failed"; exit 1; }
echo "c ok"
bash tools/gpu_r03_b.sh
