#!/bin/bash
# Round 6: the id-plan tests (distinct ids, run heads, planned sparse update), then the C3 bench line
# and its rocprofv3 kernel statistics. Usage: tools/gpu_r06_b.sh TAG [extra pytest files...]
cd "$(dirname "$0")/.."
tag=${1:-r06b}; shift
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
    tests/test_gpu_inbatch_dedup.py tests/test_gpu_c3_dedup_at_size.py "$@" > $out/tests.log 2>&1
rc=$?; tail -3 $out/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py --config c3 --extras off -o $out/c3_line.json > $out/c3_bench.log 2>&1 || exit $?
python3 -c "
import json; d = json.load(open('$out/c3_line.json')); g = d['roofline'].get('gather', {}).get('in_step', {})
print('c3', d['ms_per_step'], d['value'], d['roofline']['frac'], 'gather', g.get('avg_launch_ms'), g.get('frac'))"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $out/prof -o p -- \
    python3 bench.py --config c3 --extras off --steps 20 --warmup 3 --no-cpu-baseline --no-f32-compare \
    -o $out/c3_prof_line.json > $out/c3_prof.log 2>&1 || exit $?
f=$(find $out/prof -name "*results.db" | head -1)
python3 tools/rocpd_stats.py $f $out/c3_kernel_stats.csv 60 > $out/c3_kernel_stats.txt 2>&1
rm -rf $out/prof
head -12 $out/c3_kernel_stats.txt | cut -c1-150
