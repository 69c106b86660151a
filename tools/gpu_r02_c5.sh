#!/bin/bash
# round 2: dcn2 tests (multi-gather, planes), then the c5 bench line and its rocprof kernel stats
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -x -q -m gpu -k "${TESTS:-dcn2 or multi or planes or xgemm}" -p no:cacheprovider \
  --timeout 200 --timeout-method thread > gpurun_out/tests_c5.log 2>&1
rc=$?; tail -3 gpurun_out/tests_c5.log
if [ $rc -ne 0 ]; then grep -E "^E |FAILED|Error" gpurun_out/tests_c5.log | head -40; exit $rc; fi
timeout -k 10 400 python bench.py --config c5 --steps 10 --warmup 3 --cpu-seconds 5 -o gpurun_out/bench_c5.json > gpurun_out/bench_c5.log 2>&1 || { tail -20 gpurun_out/bench_c5.log; exit 1; }
tail -c 1200 gpurun_out/bench_c5.log
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c5 -o c5 -- \
    python3 bench.py --config c5 --steps 10 --warmup 2 --no-cpu-baseline --no-f32-compare -o gpurun_out/prof_bench_c5.json > gpurun_out/prof_c5.log 2>&1 || { tail -20 gpurun_out/prof_c5.log; exit 1; }
f=$(find gpurun_out/prof_c5 -name '*kernel_stats.csv' | head -1); python tools/kstats.py $f 40 > gpurun_out/c5_kstats.txt; cat gpurun_out/c5_kstats.txt
