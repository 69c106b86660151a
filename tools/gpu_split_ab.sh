#!/bin/bash
# split-precision in-batch kernels: parity tests, then microbench current vs a variant library
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
run() { echo "+ $*"; "$@"; local rc=$?; if [ $rc -ne 0 ]; then echo "FAILED rc=$rc"; exit $rc; fi; }
run timeout -k 10 600 python -m pytest tests/test_gpu_kernels.py -x -q -k "inbatch" > gpurun_out/split_tests.log 2>&1
tail -3 gpurun_out/split_tests.log
VAR=${VAR:-tools/_exp_inbatch_v1.so}
for v in cur var cur var; do
  if [ $v = var ]; then export RECSYS_HIP_LIB=$VAR; else unset RECSYS_HIP_LIB; fi
  echo "== $v"
  run timeout -k 10 300 python tools/microbench_inbatch_prec.py 65536 ${PRECS:-6}
done
