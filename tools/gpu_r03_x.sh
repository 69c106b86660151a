#!/bin/bash
# round 3 (session 2): bound-first top-k (A0 list scan, A1 + B threshold scans, atomic-free
# candidate slots) -- parity, then Q = 1024 timing and kernel trace
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_topk_two_phase.py tests/test_gpu_c4_shard.py -x -v --timeout 300 \
    --timeout-method thread > gpurun_out/r03_x_tests.log 2>&1
rc=$?; echo "tp tests rc=$rc"; tail -3 gpurun_out/r03_x_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
for v in "RS_TOPK_TWO_PHASE=0" "RS_TOPK_RANGE_RATIO=16" "RS_TOPK_RANGE_RATIO=8" "RS_TOPK_RANGE_RATIO=24"; do
  env $v GAUSS=1 PREC=6 timeout -k 10 200 python -u tools/microbench_topk.py 12500000 100 1024 \
      > gpurun_out/r03_x_mb_${v}.log 2>&1 || exit $?
  echo "$v: $(grep 'Q= 1024' gpurun_out/r03_x_mb_${v}.log)"
done
GAUSS=1 PREC=6 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_tp2 -o tp -- \
    python3 tools/microbench_topk.py 12500000 100 1024 > gpurun_out/r03_x_tp.log 2>&1 || exit $?
f=$(find gpurun_out/prof_tp2 -name '*kernel_stats.csv' | head -1); python3 tools/kstats.py $f 8
