#!/bin/bash
# round 4: device-count dedup tests, C2 gradient-error diagnostic, kernel trace of the c3 step (idle gaps)
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_inbatch_dedup.py -x -q --timeout 300 --timeout-method thread \
    -k "device_count or graphed" > gpurun_out/r04_d_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -5 gpurun_out/r04_d_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -u tools/diag_c2_grad_err.py > gpurun_out/r04_c_diag.log 2>&1 || exit $?
tail -32 gpurun_out/r04_c_diag.log
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_r04d -o z -- \
    python3 bench.py --extras off --no-cpu-baseline --no-f32-compare --steps 20 --warmup 3 > gpurun_out/r04_d_bench.log 2>&1 || exit $?
f=$(find gpurun_out/prof_r04d -name '*kernel_trace.csv' | head -1); cp $f gpurun_out/r04_d_trace.csv
python3 tools/trace_gaps.py gpurun_out/r04_d_trace.csv > gpurun_out/r04_d_gaps.txt 2>&1
tail -30 gpurun_out/r04_d_gaps.txt
