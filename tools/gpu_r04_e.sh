#!/bin/bash
# round 4: the GPU suite at the current tree, then smoke, C2 gradient-error diagnostic, c3 trace gaps
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/r04_e_suite.log 2>&1
rc=$?; echo "suite rc=$rc"; tail -12 gpurun_out/r04_e_suite.log
timeout -k 10 300 python -u tools/diag_c2_grad_err.py > gpurun_out/r04_c_diag.log 2>&1 || exit $?
tail -32 gpurun_out/r04_c_diag.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -c 'import __graft_entry__ as g; g.smoke()' > gpurun_out/r04_e_smoke.log 2>&1 || exit $?
tail -1 gpurun_out/r04_e_smoke.log
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_r04e -o z -- \
    python3 bench.py --extras off --no-cpu-baseline --no-f32-compare --steps 20 --warmup 3 > gpurun_out/r04_e_bench.log 2>&1 || exit $?
f=$(find gpurun_out/prof_r04e -name '*kernel_trace.csv' | head -1); cp $f gpurun_out/r04_e_trace.csv
python3 tools/trace_gaps.py gpurun_out/r04_e_trace.csv > gpurun_out/r04_e_gaps.txt 2>&1
tail -30 gpurun_out/r04_e_gaps.txt
