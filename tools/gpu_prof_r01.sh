#!/bin/bash
# round-1 profiles: top-k microbench, then rocprofv3 kernel stats of the c3 / c5 / c2 benches
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
run() { echo "+ $*"; "$@"; local rc=$?; if [ $rc -ne 0 ]; then echo "FAILED rc=$rc: $*"; exit $rc; fi; }
run timeout -k 10 400 python tools/microbench_topk.py 12500000 100 1,64,1024
for c in c3 c5 c2; do
  steps=10; [ $c = c2 ] && steps=50
  run timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$c -o $c -- \
      python3 bench.py --config $c --steps $steps --warmup 2 --no-cpu-baseline -o gpurun_out/prof_bench_$c.json
done
for c in c3 c5 c2; do f=$(find gpurun_out/prof_$c -name '*kernel_stats.csv' | head -1); echo "== $c $f"; python tools/kstats.py $f 14; done
