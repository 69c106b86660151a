#!/bin/bash
# round 3 (session 2): fused retrieval+cross node, addend prefetched in the float4 cross backward
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
    -k "dcn or cross or model or multitask or dedup" > gpurun_out/r03_fuse2_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/r03_fuse2_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
bash tools/gpu_r03_c3prof.sh > /dev/null || exit $?
grep -E "dcn_cross|Functor|inbatch_(row|col)_m16|total" gpurun_out/r03_c3_kstats.txt | cut -c1-140
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --config c3 --steps 50 --warmup 5 --no-cpu-baseline --extras off \
      --no-f32-compare -o gpurun_out/r03_fuse2_c3_$i.json > gpurun_out/r03_fuse2_c3_$i.log 2>&1 || exit $?
  python3 -c "import json;d=json.load(open('gpurun_out/r03_fuse2_c3_$i.json'));print('c3', d['ms_per_step'], d['value'], d['roofline']['frac'])"
done
