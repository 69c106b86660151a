#!/bin/bash
# A/B of two library builds on one box: $OLD (default tools/_ab_old_gemm.so) vs the in-tree one,
# twice interleaved, on the command in $CMD (default: the C3 tower microbench); then the GPU tests
# selected by $KSEL on the in-tree library.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
OLD=${OLD:-tools/_ab_old_gemm.so}
CMD=${CMD:-python tools/microbench_towers.py}
for r in 1 2; do
  for lib in $OLD recommendation-system-maang-nvidia-_amd/librecsys_hip.so; do
    echo "== $lib"
    RECSYS_HIP_LIB=$PWD/$lib timeout -k 10 200 $CMD 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
if [ -n "$KSEL" ]; then
  timeout -k 10 600 python -u -m pytest tests -x -q -m gpu -k "$KSEL" -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/ab_tests.log 2>&1; rc=$?
  tail -3 gpurun_out/ab_tests.log; exit $rc
fi
