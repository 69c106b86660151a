cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests/test_gpu_kernels.py -q -m gpu -p no:cacheprovider > gpurun_out/t1.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/t1.log
if [ $rc -le 1 ]; then
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke1.log 2>&1
  echo "smoke rc=$?" >> gpurun_out/smoke1.log
fi
tail -30 gpurun_out/t1.log
cat gpurun_out/smoke1.log 2>/dev/null | tail -20
