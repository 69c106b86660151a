#!/bin/bash
# GEMM parity tests (current library), then timing A/B of the current library vs VARS
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
run() { echo "+ $*"; "$@"; local rc=$?; if [ $rc -ne 0 ]; then echo "FAILED rc=$rc"; exit $rc; fi; }
run timeout -k 10 300 python -m pytest tests/test_gpu_kernels.py tests/test_gpu_dcn2.py tests/test_gpu_model.py -x -q -p no:cacheprovider > gpurun_out/gemm_tests.log 2>&1
tail -1 gpurun_out/gemm_tests.log
for rep in 1 2; do
  for v in cur ${VARS}; do
    if [ $v = cur ]; then unset RECSYS_HIP_LIB; else export RECSYS_HIP_LIB=tools/_exp_gemm_$v.so; fi
    echo "== $v"
    run timeout -k 10 300 python tools/microbench_gemm_prec.py ${PRECS:-6}
  done
done
