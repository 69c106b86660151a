#!/bin/bash
# round 4: the C3-size dedup parity test, the dedup microbench kernel stats, a short c3 bench line
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_c3_dedup_at_size.py -x -v --timeout 300 --timeout-method thread \
    > gpurun_out/r04_a_test.log 2>&1
rc=$?; echo "test rc=$rc"; tail -5 gpurun_out/r04_a_test.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r04a -o z -- \
    python3 tools/microbench_inbatch_dedup.py 10 > gpurun_out/r04_a_mb.log 2>&1 || exit $?
tail -2 gpurun_out/r04_a_mb.log
f=$(find gpurun_out/prof_r04a -name '*kernel_stats.csv' | head -1); python3 tools/kstats.py $f 12 > gpurun_out/r04_a_kstats.txt
head -8 gpurun_out/r04_a_kstats.txt | cut -c1-200
timeout -k 10 300 python -u bench.py --extras off --no-cpu-baseline --steps 30 -o gpurun_out/r04_a_bench.json > gpurun_out/r04_a_bench.log 2>&1 || exit $?
tail -c 600 gpurun_out/r04_a_bench.log
