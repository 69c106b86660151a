#!/bin/bash
# rocprofv3 kernel stats of the c3 / c5 / c2 benches (default precision) -> gpurun_out/prof_<c>
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
run() { echo "+ $*"; "$@"; local rc=$?; if [ $rc -ne 0 ]; then echo "FAILED rc=$rc: $*"; exit $rc; fi; }
for c in c3 c5 c2; do
  steps=10; [ $c = c2 ] && steps=50
  run timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$c -o $c -- \
      python3 bench.py --config $c --steps $steps --warmup 2 --no-cpu-baseline --no-f32-compare \
      -o gpurun_out/prof_bench_$c.json > gpurun_out/prof_$c.log 2>&1
done
for c in c3 c5 c2; do f=$(find gpurun_out/prof_$c -name '*kernel_stats.csv' | head -1); echo "== $c"; python tools/kstats.py $f 12; done
