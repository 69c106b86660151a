#!/bin/bash
# round 4: the one-launch Dense stack kernels (rs_mlp_*) reading pre-split weight fragment images:
# the microbench, their tests at both row counts + the model tests, then c2 lines (off / 32 / 16
# rows) and the c2 kernel stats
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 python3 tools/microbench_mlp.py 2>&1 | grep -v amdgpu.ids || exit 1
for r in 16 32; do
  RS_MLP_ROWS=$r timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q --timeout 120 \
      --timeout-method thread -k "mlp or tower or gemm_group" > gpurun_out/r04_w_tests_$r.log 2>&1
  rc=$?; echo "mlp tests rows=$r rc=$rc"; tail -2 gpurun_out/r04_w_tests_$r.log; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 400 python -u -m pytest tests/test_gpu_model.py tests/test_gpu_dcn2.py -m gpu -x -q --timeout 300 \
    --timeout-method thread > gpurun_out/r04_w_tests_model.log 2>&1
rc=$?; echo "model tests rc=$rc"; tail -2 gpurun_out/r04_w_tests_model.log; [ $rc -eq 0 ] || exit $rc
for v in "0 16" "16384 16" "16384 32" "0 16" "16384 16" "16384 32"; do
  set -- $v
  RS_MLP_FUSED_MAX_M=$1 RS_MLP_ROWS=$2 timeout -k 10 300 python -u bench.py --config c2 --extras off --no-cpu-baseline \
      --no-f32-compare --steps 100 -o gpurun_out/r04_w_c2_$1_$2.json > gpurun_out/r04_w_c2_$1_$2.log 2>&1 || exit $?
  python3 -c "import json; d=json.load(open('gpurun_out/r04_w_c2_$1_$2.json')); print('c2 fused<=$1 rows=$2', d['ms_per_step'], d['value'])"
done
for r in 16 32; do
  RS_MLP_ROWS=$r timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_w$r -o c2 -- python3 bench.py \
      --config c2 --extras off --no-cpu-baseline --no-f32-compare --steps 20 --eager > gpurun_out/r04_w_prof$r.log 2>&1 || exit $?
  f=$(find gpurun_out/prof_w$r -name "*results.db" | head -1)
  python3 tools/rocpd_stats.py $f gpurun_out/r04_w_c2_kernel_stats_$r.csv 40 > gpurun_out/r04_w_c2_kernel_stats_$r.txt 2>&1
  rm -rf gpurun_out/prof_w$r
  echo "rows=$r"; head -8 gpurun_out/r04_w_c2_kernel_stats_$r.txt | cut -c1-130
done
