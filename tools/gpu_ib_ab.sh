#!/bin/bash
# A/B of in-batch kernel variants: for the current library and each tools/_exp_inbatch_<v>.so
# (VARS="a b ..."): the in-batch parity tests, then the precision microbench (with bitwise
# checksums of lse / dU / dC / S), twice, interleaved
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
run() { echo "+ $*"; "$@"; local rc=$?; if [ $rc -ne 0 ]; then echo "FAILED rc=$rc"; exit $rc; fi; }
for v in ${VARS}; do
  export RECSYS_HIP_LIB=tools/_exp_inbatch_$v.so
  run timeout -k 10 300 python -m pytest tests/test_gpu_kernels.py tests/test_gpu_model.py -x -q -k "inbatch" -p no:cacheprovider > gpurun_out/ib_tests_$v.log 2>&1
  tail -1 gpurun_out/ib_tests_$v.log
done
for rep in 1 2; do
  for v in cur ${VARS}; do
    if [ $v = cur ]; then unset RECSYS_HIP_LIB; else export RECSYS_HIP_LIB=tools/_exp_inbatch_$v.so; fi
    echo "== $v"
    run timeout -k 10 300 python tools/microbench_inbatch_prec.py 65536 ${PRECS:-6}
  done
done
