#!/bin/bash
# round 3 (session 2): smoke(), then the c2 graphed line and its kernel trace at the final code
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r03_smoke.log 2>&1 || exit $?
tail -1 gpurun_out/r03_smoke.log
timeout -k 10 200 python -u bench.py --config c2 --steps 300 --warmup 20 --no-cpu-baseline --extras off \
    --no-f32-compare -o gpurun_out/r03_c2final.json > gpurun_out/r03_c2final.log 2>&1 || exit $?
python3 -c "import json;d=json.load(open('gpurun_out/r03_c2final.json'));print('c2', d['ms_per_step'], d['value'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c2f -o c2 -- \
    python3 bench.py --config c2 --steps 100 --warmup 10 --no-cpu-baseline --extras off --no-f32-compare \
    -o gpurun_out/r03_c2final_prof.json > gpurun_out/r03_c2final_prof.log 2>&1 || exit $?
f=$(find gpurun_out/prof_c2f -name '*kernel_stats.csv' | head -1); python3 tools/kstats.py $f 60 > gpurun_out/r03_c2final_kstats.txt
tail -1 gpurun_out/r03_c2final_kstats.txt
