#!/bin/bash
# full GPU test suite (one pytest process) + smoke
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -q -m gpu -p no:cacheprovider > gpurun_out/tests.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/tests.log
tail -25 gpurun_out/tests.log
if [ $rc -le 1 ]; then
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" 2>&1 | grep -v amdgpu.ids
fi
