#!/bin/bash
# round 3 (session 2): 8-wave 64-row-tile threshold scan as default -- top-k parity, c4 PMC traffic, c4 line
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_topk_two_phase.py tests/test_gpu_c4_shard.py tests/test_gpu_kernels.py \
    -k "topk or shard or two_phase" -x -q --timeout 300 --timeout-method thread > gpurun_out/r03_w8c_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/r03_w8c_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
d=gpurun_out/pmc_c4w8
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 150 rocprofv3 --kernel-trace --pmc $c --output-format csv -d $d/$c -o x -- \
      python3 tools/traffic_probe.py c4 4 > $d.$c.log 2>&1 || { echo "pmc $c failed"; exit 1; }
done
python3 tools/traffic_summary.py gpurun_out/r03_pmc_c4_w8.json c4=$d:4
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c4w8 -o c4 -- \
    python3 bench.py --config c4 --steps 10 --warmup 2 -o gpurun_out/r03_w8c_c4.json > gpurun_out/r03_w8c_c4.log 2>&1 || exit $?
f=$(find gpurun_out/prof_c4w8 -name '*kernel_stats.csv' | head -1); python3 tools/kstats.py $f 20 > gpurun_out/r03_c4w8_kstats.txt
head -4 gpurun_out/r03_c4w8_kstats.txt | cut -c1-150
python3 -c "import json;d=json.load(open('gpurun_out/r03_w8c_c4.json'));print('c4', d['ms_per_step'], d['roofline'])"
