#!/bin/bash
# bench (c3 and c2) + rocprofv3 kernel trace of the c3 bench; outputs under gpurun_out/
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python bench.py --steps 10 --warmup 3 > gpurun_out/bench_c3.json 2> gpurun_out/bench_c3.err
rc=$?; echo "bench c3 rc=$rc"; tail -3 gpurun_out/bench_c3.err; cat gpurun_out/bench_c3.json
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --config c2 --steps 50 --warmup 5 --no-cpu-baseline > gpurun_out/bench_c2.json 2> gpurun_out/bench_c2.err
rc=$?; echo "bench c2 rc=$rc"; cat gpurun_out/bench_c2.json
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c3 -o c3 -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/prof_c3.log 2>&1
rc=$?; echo "rocprof rc=$rc"; tail -5 gpurun_out/prof_c3.log
find gpurun_out/prof_c3 -name "*stats*" | head
