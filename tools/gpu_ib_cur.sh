#!/bin/bash
# in-batch parity tests + precision microbench of the current library (twice)
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
run() { echo "+ $*"; "$@"; local rc=$?; if [ $rc -ne 0 ]; then echo "FAILED rc=$rc"; exit $rc; fi; }
run timeout -k 10 300 python -m pytest tests/test_gpu_kernels.py tests/test_gpu_model.py -x -q -k "inbatch" -p no:cacheprovider > gpurun_out/ib_tests_cur.log 2>&1
tail -1 gpurun_out/ib_tests_cur.log
for rep in 1 2; do run timeout -k 10 300 python tools/microbench_inbatch_prec.py 65536 ${PRECS:-6}; done
