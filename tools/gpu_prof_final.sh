#!/bin/bash
# round-end evidence: rocprofv3 kernel stats of the c3 / c5 / c2 / c4 benches, MFMA busy of the
# split GEMMs (c5 shapes), then the default bench line with its CPU baseline
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
run() { echo "+ $*"; "$@"; local rc=$?; if [ $rc -ne 0 ]; then echo "FAILED rc=$rc: $*"; exit $rc; fi; }
for c in c3 c5 c2 c4; do
  steps=10; [ $c = c2 ] && steps=50; [ $c = c4 ] && steps=5
  run timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$c -o $c -- \
      python3 bench.py --config $c --steps $steps --warmup 2 --no-cpu-baseline --no-f32-compare -o gpurun_out/prof_bench_$c.json
done
for c in c3 c5 c2 c4; do f=$(find gpurun_out/prof_$c -name '*kernel_stats.csv' | head -1); echo "== $c $f"; python tools/kstats.py $f 14; done
run bash tools/gpu_pmc_gemm_x3.sh > gpurun_out/pmc_x3.log 2>&1
run timeout -k 10 900 python bench.py -o gpurun_out/bench_default.json
