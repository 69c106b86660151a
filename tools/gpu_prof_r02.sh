#!/bin/bash
# round-2 profiles: the whole GPU test suite, rocprofv3 kernel stats of the c2 / c3 /
# c4 / c5 benches, then the default c3 bench line (with its CPU baseline) for profiles/
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
run() { echo "+ $*"; "$@"; local rc=$?; if [ $rc -ne 0 ]; then echo "FAILED rc=$rc: $*"; exit $rc; fi; }
run timeout -k 10 600 python -u -m pytest tests -x -q -m gpu -p no:cacheprovider \
    --timeout 120 --timeout-method thread
for c in c2 c3 c4 c5; do
  steps=10; [ $c = c2 ] && steps=50; [ $c = c4 ] && steps=5
  run timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$c -o $c -- \
      python3 bench.py --config $c --steps $steps --warmup 2 --no-cpu-baseline --no-f32-compare \
      -o gpurun_out/prof_bench_$c.json
done
for c in c2 c3 c4 c5; do
  f=$(find gpurun_out/prof_$c -name '*kernel_stats.csv' | head -1); cp $f gpurun_out/r02_${c}_kernel_stats.csv
  python tools/kstats.py $f 40 > gpurun_out/r02_${c}_kernel_stats.txt; echo "== $c"; head -8 gpurun_out/r02_${c}_kernel_stats.txt
done
run timeout -k 10 600 python bench.py -o gpurun_out/r02_c3_bench_line.json
