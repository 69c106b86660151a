#!/bin/bash
# round 4: the one-launch Dense stack forward / input-gradient chain / weight gradients
# (rs_mlp_*): the kernel, model and size tests, then c2 lines with them off / on, a c3 line, and
# the c2 kernel stats
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 800 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_model.py tests/test_gpu_dcn2.py \
    tests/test_gpu_inbatch_dedup.py tests/test_gpu_c3_dedup_at_size.py tests/test_gpu_production_sizes.py \
    -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r04_t_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r04_t_tests.log; [ $rc -eq 0 ] || exit $rc
SKIP_TESTS=1 bash tools/gpu_r04_s.sh || exit $?
timeout -k 10 300 python -u bench.py --config c3 --extras off --no-cpu-baseline --no-f32-compare --steps 40 \
    -o gpurun_out/r04_t_c3.json > gpurun_out/r04_t_c3.log 2>&1 || exit $?
python3 -c "import json; d=json.load(open('gpurun_out/r04_t_c3.json')); print('c3', d['ms_per_step'], d['value'], d['roofline']['frac'])"
