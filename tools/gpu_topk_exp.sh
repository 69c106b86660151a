#!/bin/bash
# timing-only top-k experiment variants (tools/_exp_topk_<v>.so), Q list in QS
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
run() { echo "+ $*"; "$@"; local rc=$?; if [ $rc -ne 0 ]; then echo "FAILED rc=$rc"; exit $rc; fi; }
for rep in 1 2; do
  for v in cur ${VARS}; do
    if [ $v = cur ]; then unset RECSYS_HIP_LIB; else export RECSYS_HIP_LIB=tools/_exp_topk_$v.so; fi
    echo "== $v"
    run timeout -k 10 300 python tools/microbench_topk.py 12500000 100 ${QS:-1024}
  done
done
