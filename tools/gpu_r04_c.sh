#!/bin/bash
# round 4: C2 gradient-error diagnostic (precision 6 / 0 / 9 vs float64 under the GPU's gates)
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/diag_c2_grad_err.py > gpurun_out/r04_c_diag.log 2>&1 || exit $?
cat gpurun_out/r04_c_diag.log | tail -32
