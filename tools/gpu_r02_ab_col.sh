#!/bin/bash
# A/B of the stored col pass: tools/_ab_old_lib.so (before) against the in-tree library (after),
# interleaved, C3 in-batch pair at B = 65536, precision 6; then the in-batch GPU parity tests.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for r in 1 2; do
  for lib in tools/_ab_old_lib.so recommendation-system-maang-nvidia-_amd/librecsys_hip.so; do
    echo "== $lib"
    RECSYS_HIP_LIB=$PWD/$lib timeout -k 10 120 python tools/microbench_inbatch_prec.py 65536 6 || exit 1
  done
done
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu -k "inbatch" -p no:cacheprovider --timeout 300 --timeout-method thread
