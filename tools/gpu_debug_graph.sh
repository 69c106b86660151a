#!/bin/bash
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -X faulthandler bench.py --config c2 --steps 20 --warmup 2 --no-cpu-baseline > gpurun_out/dbg.json 2> gpurun_out/dbg.err
rc=$?
echo "rc=$rc"
grep -v amdgpu.ids gpurun_out/dbg.err | tail -40
exit $rc
