#!/bin/bash
# The driver's default bench line, the C2 line, then the default command under
# rocprofv3 --kernel-trace --stats (kernel statistics -> TAG_c3_kernel_stats.txt) and the C2 one.
cd "$(dirname "$0")/.."
TAG=${1:-run}   # output prefix, e.g. r05
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u bench.py -o gpurun_out/${TAG}_bench_default_line.json > gpurun_out/${TAG}_bench.log 2>&1 || exit $?
timeout -k 10 600 python -u bench.py --config c2 -o gpurun_out/${TAG}_c2_line.json > gpurun_out/${TAG}_c2_bench.log 2>&1 || exit $?
python3 -c "
import json
for f in ('${TAG}_bench_default_line', '${TAG}_c2_line'):
    d = json.load(open('gpurun_out/%s.json' % f)); print(f, d['ms_per_step'], d['value'], d['roofline']['frac'])"
for c in c3 c2; do
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$c -o p -- \
      python3 bench.py --config $c --extras off --steps 20 --warmup 3 --no-cpu-baseline \
      -o gpurun_out/${TAG}_${c}_bench_prof.json > gpurun_out/${TAG}_${c}_prof.log 2>&1 || exit $?
  f=$(find gpurun_out/prof_$c -name "*results.db" | head -1)
  python3 tools/rocpd_stats.py $f gpurun_out/${TAG}_${c}_kernel_stats.csv 60 > gpurun_out/${TAG}_${c}_kernel_stats.txt 2>&1
  rm -rf gpurun_out/prof_$c
  head -6 gpurun_out/${TAG}_${c}_kernel_stats.txt | cut -c1-150
done
