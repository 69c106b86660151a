#!/bin/bash
# round 4: the driver's default bench line (all sub-records), then its kernel stats
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u bench.py -o gpurun_out/r04_l_bench.json > gpurun_out/r04_l_bench.log 2>&1 || exit $?
python3 -c "import json; d=json.load(open('gpurun_out/r04_l_bench.json')); print(d['ms_per_step'], d['value'], d['roofline']['frac'])"
