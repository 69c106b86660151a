#!/bin/bash
# kernel-level split of the top-k (scan vs merge) under rocprofv3
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
run() { echo "+ $*"; "$@"; local rc=$?; if [ $rc -ne 0 ]; then echo "FAILED rc=$rc: $*"; exit $rc; fi; }
for Q in ${QS:-16 1024}; do
  run timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_topk_$Q -o t -- \
      python3 tools/microbench_topk.py 12500000 100 $Q
  f=$(find gpurun_out/prof_topk_$Q -name '*kernel_stats.csv' | head -1); python tools/kstats.py $f 8
done
