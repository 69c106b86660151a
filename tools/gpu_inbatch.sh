#!/bin/bash
# in-batch parity (incl. stored-scores == recompute), microbench, then the c3 bench
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
run() { echo "+ $*"; "$@"; local rc=$?; if [ $rc -ne 0 ]; then echo "FAILED rc=$rc: $*"; exit $rc; fi; }
timeout -k 10 600 python -m pytest tests/test_gpu_kernels.py tests/test_gpu_model.py -q -m gpu -k "inbatch or oracle or graph or determin" -p no:cacheprovider > gpurun_out/t_inb.log 2>&1
rc=$?; tail -3 gpurun_out/t_inb.log
if [ $rc -ne 0 ]; then grep -E "^E |FAILED" gpurun_out/t_inb.log | head -30; exit $rc; fi
run timeout -k 10 300 python tools/microbench_inbatch.py 65536 128
run timeout -k 10 600 python bench.py --steps 10 --warmup 3 --no-cpu-baseline -o gpurun_out/bench_c3.json
