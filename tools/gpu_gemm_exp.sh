#!/bin/bash
# timing-only GEMM experiment variants (results not checked)
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
run() { echo "+ $*"; "$@"; local rc=$?; if [ $rc -ne 0 ]; then echo "FAILED rc=$rc"; exit $rc; fi; }
for rep in 1 2; do
  for v in cur ${VARS}; do
    if [ $v = cur ]; then unset RECSYS_HIP_LIB; else export RECSYS_HIP_LIB=tools/_exp_gemm_$v.so; fi
    echo "== $v"
    run timeout -k 10 300 python tools/microbench_gemm_prec.py ${PRECS:-6}
  done
done
