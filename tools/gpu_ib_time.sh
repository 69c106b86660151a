#!/bin/bash
# timing-only A/B of in-batch variants (no parity: probe builds compute wrong values)
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
for rep in 1 2; do
  for v in cur ${VARS}; do
    if [ $v = cur ]; then unset RECSYS_HIP_LIB; else export RECSYS_HIP_LIB=tools/_exp_inbatch_$v.so; fi
    echo "== $v"
    timeout -k 10 300 python tools/microbench_inbatch_prec.py 65536 ${PRECS:-6} || exit 1
  done
done
