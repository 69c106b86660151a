#!/bin/bash
# PMC traffic passes (one counter group per pass, kernel-trace only) + microbenches
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python tools/microbench_gather.py 2>&1 | grep -v amdgpu.ids
timeout -k 10 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch -o ib -- python3 tools/microbench_inbatch.py 65536 128 > gpurun_out/pmc_fetch.log 2>&1
echo "pmc fetch rc=$?"
timeout -k 10 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write -o ib -- python3 tools/microbench_inbatch.py 65536 128 > gpurun_out/pmc_write.log 2>&1
echo "pmc write rc=$?"
timeout -k 10 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_gfetch -o g -- python3 tools/microbench_gather.py 65536 1048576 > gpurun_out/pmc_gfetch.log 2>&1
echo "pmc gather fetch rc=$?"
timeout -k 10 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_gwrite -o g -- python3 tools/microbench_gather.py 65536 1048576 > gpurun_out/pmc_gwrite.log 2>&1
echo "pmc gather write rc=$?"
ls gpurun_out/pmc_fetch gpurun_out/pmc_write
