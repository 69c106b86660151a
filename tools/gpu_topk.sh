#!/bin/bash
# top-k parity tests, then the C4 shard microbench (product lib + experiment variants)
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
run() { echo "+ $*"; "$@"; local rc=$?; if [ $rc -ne 0 ]; then echo "FAILED rc=$rc: $*"; exit $rc; fi; }
timeout -k 10 600 python -m pytest tests/test_gpu_kernels.py -q -m gpu -k topk -p no:cacheprovider > gpurun_out/t_topk.log 2>&1
rc=$?; tail -4 gpurun_out/t_topk.log
if [ $rc -ne 0 ]; then grep -E "^E |FAILED" gpurun_out/t_topk.log | head -30; exit $rc; fi
run timeout -k 10 400 python tools/microbench_topk.py 12500000 100 1,16,64,1024
for v in ${TOPK_VARIANTS:-}; do
  echo "== variant $v"
  RECSYS_HIP_LIB=$PWD/tools/_exp_topk_$v.so run timeout -k 10 400 python tools/microbench_topk.py 12500000 100 1,16,64,1024
done
