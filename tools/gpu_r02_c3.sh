#!/bin/bash
# round 2: gather/embedding GPU tests, the c3 bench line, then rocprofv3 kernel stats of the c3 bench
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -x -q -m gpu -k "${TESTS:-gather or embedding or sparse}" -p no:cacheprovider \
  --timeout 120 --timeout-method thread > gpurun_out/tests_c3.log 2>&1
rc=$?; tail -3 gpurun_out/tests_c3.log
if [ $rc -ne 0 ]; then grep -E "^E |FAILED|Error" gpurun_out/tests_c3.log | head -40; exit $rc; fi
timeout -k 10 600 python bench.py --steps 20 --warmup 3 --cpu-seconds 10 -o gpurun_out/bench_c3.json > gpurun_out/bench_c3.log 2>&1 || { tail -20 gpurun_out/bench_c3.log; exit 1; }
tail -c 2500 gpurun_out/bench_c3.log
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c3 -o c3 -- \
    python3 bench.py --config c3 --steps 10 --warmup 2 --no-cpu-baseline --no-f32-compare -o gpurun_out/prof_bench_c3.json > gpurun_out/prof_c3.log 2>&1 || { tail -20 gpurun_out/prof_c3.log; exit 1; }
f=$(find gpurun_out/prof_c3 -name '*kernel_stats.csv' | head -1); python tools/kstats.py $f 30 > gpurun_out/c3_kstats.txt; cat gpurun_out/c3_kstats.txt
