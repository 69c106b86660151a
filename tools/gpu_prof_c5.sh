#!/bin/bash
# rocprofv3 kernel stats of the c5 bench (arg 1 = tag)
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${1:-c5}
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$tag -o $tag -- \
    python3 bench.py --config c5 --steps 10 --warmup 2 --no-cpu-baseline --no-f32-compare -o gpurun_out/prof_bench_$tag.json > gpurun_out/prof_$tag.log 2>&1
rc=$?
f=$(find gpurun_out/prof_$tag -name '*kernel_stats.csv' | head -1)
echo "== $tag $f"; python tools/kstats.py $f 22
tail -c 1500 gpurun_out/prof_bench_$tag.json
exit $rc
