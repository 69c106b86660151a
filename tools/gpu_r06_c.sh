#!/bin/bash
# Round 6: LDS-DMA dW kernel + planned sparse apply. Tests, then A/B (variants/wgws.so = the round-5
# wgrad_ws_kernel) on the towers microbench and the C3 step, the release build's kernel statistics,
# and the data-parallel sparse costs. Usage: tools/gpu_r06_c.sh TAG
cd "$(dirname "$0")/.."
tag=${1:-r06c}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
rel=recommendation-system-maang-nvidia-_amd/librecsys_hip.so
timeout -k 10 700 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
    tests/test_gpu_kernels.py -k "wgrad or gemm_group or mlp" > $out/tests_k.log 2>&1
rc=$?; tail -3 $out/tests_k.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
    tests/test_gpu_inbatch_dedup.py tests/test_gpu_c3_dedup_at_size.py > $out/tests_d.log 2>&1
rc=$?; tail -3 $out/tests_d.log; [ $rc -eq 0 ] || exit $rc
for lib in variants/wgws.so $rel; do
  RECSYS_HIP_LIB=$lib timeout -k 10 300 python -u tools/microbench_towers.py > $out/towers_$(basename $lib .so).log 2>&1 || exit $?
  tail -6 $out/towers_$(basename $lib .so).log
done
for rep in 1 2; do
  for lib in variants/wgws.so $rel; do
    t=$(basename $lib .so)
    RECSYS_HIP_LIB=$lib timeout -k 10 300 python -u bench.py --config c3 --extras off --steps 30 --no-cpu-baseline \
        --no-f32-compare -o $out/c3_${t}_$rep.json > $out/c3_${t}_$rep.log 2>&1 || exit $?
    python3 -c "import json; d=json.load(open('$out/c3_${t}_$rep.json')); print('$t', d['ms_per_step'], d['roofline']['frac'])"
  done
done
timeout -k 10 300 python -u tools/microbench_dp_sparse.py 8 > $out/dp_sparse.log 2>&1 || exit $?
tail -1 $out/dp_sparse.log
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $out/prof -o p -- \
    python3 bench.py --config c3 --extras off --steps 20 --warmup 3 --no-cpu-baseline --no-f32-compare \
    -o $out/c3_prof_line.json > $out/c3_prof.log 2>&1 || exit $?
f=$(find $out/prof -name "*results.db" | head -1)
python3 tools/rocpd_stats.py $f $out/c3_kernel_stats.csv 60 > $out/c3_kernel_stats.txt 2>&1
rm -rf $out/prof
head -14 $out/c3_kernel_stats.txt | cut -c1-150
