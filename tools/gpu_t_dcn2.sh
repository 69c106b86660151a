#!/bin/bash
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_dcn2.py tests/test_gpu_kernels.py -q -m gpu -p no:cacheprovider > gpurun_out/t_dcn2.log 2>&1
rc=$?; tail -4 gpurun_out/t_dcn2.log
if [ $rc -ne 0 ]; then grep -E "^E |FAILED|Error" gpurun_out/t_dcn2.log | head -40; fi
exit $rc
