#!/bin/bash
# round 4: the one-launch Dense stack forward (rs_mlp_fwd_prec_f32): its tests and the model tests,
# then c2 lines with it off / on, and the c2 kernel stats
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
[ -n "$SKIP_TESTS" ] || { timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_model.py tests/test_gpu_dcn2.py \
    -m gpu -x -q --timeout 300 --timeout-method thread -k "mlp or tower or model or dcn or heads" \
    > gpurun_out/r04_s_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r04_s_tests.log; [ $rc -eq 0 ] || exit $rc; }
for v in 0 16384 0 16384; do
  RS_MLP_FUSED_MAX_M=$v timeout -k 10 300 python -u bench.py --config c2 --extras off --no-cpu-baseline \
      --no-f32-compare --steps 100 -o gpurun_out/r04_s_c2_$v.json > gpurun_out/r04_s_c2_$v.log 2>&1 || exit $?
  python3 -c "import json; d=json.load(open('gpurun_out/r04_s_c2_$v.json')); print('c2 fused<=$v', d['ms_per_step'], d['value'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_s -o c2 -- python3 bench.py --config c2 \
    --extras off --no-cpu-baseline --no-f32-compare --steps 20 --eager > gpurun_out/r04_s_prof.log 2>&1 || exit $?
f=$(find gpurun_out/prof_s -name "*results.db" | head -1)
python3 tools/rocpd_stats.py $f gpurun_out/r04_s_c2_kernel_stats.csv 40 > gpurun_out/r04_s_c2_kernel_stats.txt 2>&1
rm -rf gpurun_out/prof_s
head -25 gpurun_out/r04_s_c2_kernel_stats.txt | cut -c1-150
