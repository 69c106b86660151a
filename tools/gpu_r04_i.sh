#!/bin/bash
# round 4: where the time goes now — c2 and c5 lines + kernel stats (rocprofv3), c3 graphed stats
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
for c in c2 c5; do
  timeout -k 10 300 python -u bench.py --config $c --extras off --no-cpu-baseline --no-f32-compare --steps 30 \
      -o gpurun_out/r04_i_$c.json > gpurun_out/r04_i_$c.log 2>&1 || exit $?
  python3 -c "import json; d=json.load(open('gpurun_out/r04_i_$c.json')); print('$c', d['ms_per_step'], d['value'], d['roofline']['frac'])"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r04i_$c -o p -- \
      python3 bench.py --config $c --extras off --no-cpu-baseline --no-f32-compare --steps 20 --warmup 3 > gpurun_out/r04_i_${c}_prof.log 2>&1 || exit $?
  f=$(find gpurun_out/prof_r04i_$c -name "*results.db" | head -1)
  python3 tools/rocpd_stats.py $f gpurun_out/r04_i_${c}_kstats.csv 40 > gpurun_out/r04_i_${c}_kstats.txt 2>&1; rm -rf gpurun_out/prof_r04i_$c
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r04i_c3 -o p -- \
    python3 bench.py --extras off --no-cpu-baseline --no-f32-compare --steps 20 --warmup 3 > gpurun_out/r04_i_c3_prof.log 2>&1 || exit $?
f=$(find gpurun_out/prof_r04i_c3 -name "*results.db" | head -1)
python3 tools/rocpd_stats.py $f gpurun_out/r04_i_c3_kstats.csv 40 > gpurun_out/r04_i_c3_kstats.txt 2>&1; rm -rf gpurun_out/prof_r04i_c3
echo done
