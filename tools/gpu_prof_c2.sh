#!/bin/bash
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c2 -o c2 -- python3 bench.py --config c2 --steps 20 --warmup 2 --no-cpu-baseline --eager > gpurun_out/prof_c2.log 2>&1
echo "rc=$?"
