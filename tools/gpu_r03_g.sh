#!/bin/bash
# round 3: the whole GPU suite as the driver runs it, smoke(), the default bench line, then the
# per-config kernel statistics (rocpd databases; tools/rocpd_stats.py summarises them)
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1200 python -u -m pytest tests -x -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread \
    > gpurun_out/r03_gpu_suite.log 2>&1
rc=$?; echo "suite rc=$rc"; tail -3 gpurun_out/r03_gpu_suite.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03_smoke.log 2>&1 || exit $?
echo "smoke ok"
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 -o gpurun_out/r03_bench2.json > gpurun_out/r03_bench2.log 2>&1 || exit $?
echo "bench ok"
for c in c3 c5 c4; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r03b_$c -o run -- \
      python3 bench.py --config $c --steps 10 --warmup 3 --no-cpu-baseline --no-f32-compare --extras off \
      -o gpurun_out/prof_r03b_$c.json > gpurun_out/prof_r03b_$c.log 2>&1 || { echo "prof $c failed"; exit 1; }
done
echo "prof ok"
