#!/bin/bash
# round 4: the sparse update taking the id plan's order (RS_SPARSE_PLAN_ORDER): the bitwise tests,
# the graphed-step and model tests, then c3 / c2 lines with it off / on and the c3 kernel stats
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_inbatch_dedup.py tests/test_gpu_model.py \
    -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r04_po_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -1 gpurun_out/r04_po_tests.log; [ $rc -eq 0 ] || exit $rc
for c in c3 c2; do
  for v in 0 1 0 1; do
    RS_SPARSE_PLAN_ORDER=$v timeout -k 10 300 python -u bench.py --config $c --extras off --no-cpu-baseline \
        --no-f32-compare --steps 40 -o gpurun_out/r04_po_${c}_$v.json > gpurun_out/r04_po_${c}_$v.log 2>&1 || exit $?
    python3 -c "import json; d=json.load(open('gpurun_out/r04_po_${c}_$v.json')); print('$c plan_order=$v', d['ms_per_step'], d['value'], d['roofline']['frac'])"
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_po -o c3 -- python3 bench.py \
    --extras off --no-cpu-baseline --no-f32-compare --steps 20 --warmup 3 -o gpurun_out/r04_po_prof.json \
    > gpurun_out/r04_po_prof.log 2>&1 || exit $?
f=$(find gpurun_out/prof_po -name "*results.db" | head -1)
python3 tools/rocpd_stats.py $f gpurun_out/r04_po_c3_kernel_stats.csv 60 > gpurun_out/r04_po_c3_kernel_stats.txt 2>&1
rm -rf gpurun_out/prof_po
grep -E "rocprim|sort|sparse" gpurun_out/r04_po_c3_kernel_stats.txt | cut -c1-130
