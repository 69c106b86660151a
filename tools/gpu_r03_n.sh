#!/bin/bash
# round 3: stream-K deduplicated pair -- its tests, then the c3 line and kernel statistics
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_inbatch_dedup.py -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/r03_dedup_tests2.log 2>&1
rc=$?; echo "dedup tests rc=$rc"
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r03_c3sk -o run -- \
    python3 bench.py --config c3 --steps 20 --warmup 3 --no-cpu-baseline --no-f32-compare --extras off \
    -o gpurun_out/prof_r03_c3sk.json > gpurun_out/prof_r03_c3sk.log 2>&1 || exit $?
echo "prof ok"
