#!/bin/bash
# split-precision in-batch kernels: parity tests, then the microbench for the current library and
# each variant library tools/_exp_inbatch_<v>.so (VARS="a b ..."), twice, interleaved
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
run() { echo "+ $*"; "$@"; local rc=$?; if [ $rc -ne 0 ]; then echo "FAILED rc=$rc"; exit $rc; fi; }
run timeout -k 10 600 python -m pytest tests/test_gpu_kernels.py -x -q -k "inbatch" > gpurun_out/split_tests.log 2>&1
tail -1 gpurun_out/split_tests.log
for rep in 1 2; do
  for v in cur ${VARS:-old}; do
    if [ $v = cur ]; then unset RECSYS_HIP_LIB; else export RECSYS_HIP_LIB=tools/_exp_inbatch_$v.so; fi
    echo "== $v"
    run timeout -k 10 300 python tools/microbench_inbatch_prec.py 65536 ${PRECS:-6}
  done
done
