#!/bin/bash
# c4 bench (exact top-100 over a 12.5M-row shard) and its rocprofv3 kernel stats
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
run() { echo "+ $*"; "$@"; local rc=$?; if [ $rc -ne 0 ]; then echo "FAILED rc=$rc: $*"; exit $rc; fi; }
run timeout -k 10 300 python bench.py --config c4 --steps 10 --warmup 2 -o gpurun_out/bench_c4.json
run timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c4 -o c4 -- \
    python3 bench.py --config c4 --steps 10 --warmup 2 --no-cpu-baseline
f=$(find gpurun_out/prof_c4 -name '*kernel_stats.csv' | head -1); python tools/kstats.py $f 8
