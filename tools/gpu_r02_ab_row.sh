#!/bin/bash
# A/B of the in-batch row pass: the unpipelined kernel (tools/_exp_inbatch_old.so) against the
# software-pipelined variants, C3 pair at B = 65536, precision 6 (bitsums must agree); then the
# in-batch GPU parity tests on the in-tree library.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for lib in ${BASE_LIB:-tools/_exp_inbatch_old.so} recommendation-system-maang-nvidia-_amd/librecsys_hip.so ${EXTRA_LIBS}; do
  echo "== $lib"
  RECSYS_HIP_LIB=$PWD/$lib timeout -k 10 150 python tools/microbench_inbatch_prec.py 65536 6 || exit 1
done
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu -k "inbatch" -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/ab_row_tests.log 2>&1; rc=$?
tail -3 gpurun_out/ab_row_tests.log; exit $rc
