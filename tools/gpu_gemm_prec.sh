#!/bin/bash
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
run() { echo "+ $*"; "$@"; local rc=$?; if [ $rc -ne 0 ]; then echo "FAILED rc=$rc"; exit $rc; fi; }
run timeout -k 10 600 python -m pytest tests/test_gpu_kernels.py -x -q -k "gemm" > gpurun_out/gemm_tests.log 2>&1
tail -1 gpurun_out/gemm_tests.log
run timeout -k 10 300 python tools/microbench_gemm_prec.py 0,6,9
