#!/bin/bash
# round 2: plane-GEMM tile variants (RS_PGEMM_BM = default 128 / 256 / 2564) on the c5 cross stack:
# bitwise tests under each variant, then the stack microbench
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in 2564 256; do
  RS_PGEMM_BM=$v timeout -k 10 300 python -u -m pytest tests -x -q -m gpu -k "planes" -p no:cacheprovider \
    --timeout 120 --timeout-method thread > gpurun_out/tests_pgemm_$v.log 2>&1
  rc=$?; tail -2 gpurun_out/tests_pgemm_$v.log
  if [ $rc -ne 0 ]; then grep -E "^E |FAILED|Error" gpurun_out/tests_pgemm_$v.log | head -30; exit $rc; fi
done
for v in 0 2564 256; do
  RS_PGEMM_BM=$v timeout -k 10 300 python -u tools/microbench_dcn2_planes.py 16384 > gpurun_out/pgemm_$v.log 2>&1 || exit $?
  cat gpurun_out/pgemm_$v.log
done
RS_PGEMM_BM=2564 timeout -k 10 300 python -u tools/microbench_dcn2_planes.py 65536 > gpurun_out/pgemm_2564_64k.log 2>&1 || exit $?
cat gpurun_out/pgemm_2564_64k.log
