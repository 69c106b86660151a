#!/bin/bash
# round 2: xgemm / DCN-v2 planes tests, the GEMM microbench, then the c5 bench line
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -x -q -m gpu -k "xgemm or planes or dcn2 or cross_mat" -p no:cacheprovider \
  --timeout 200 --timeout-method thread > gpurun_out/tests_xgemm.log 2>&1
rc=$?; tail -3 gpurun_out/tests_xgemm.log
if [ $rc -ne 0 ]; then grep -E "^E |FAILED|Error" gpurun_out/tests_xgemm.log | head -40; exit $rc; fi
timeout -k 10 300 python -u tools/microbench_xgemm.py 16384 > gpurun_out/xgemm_16k.log 2>&1 || exit $?
tail -4 gpurun_out/xgemm_16k.log
timeout -k 10 300 python -u tools/microbench_dcn2_planes.py 16384 > gpurun_out/dcn2_planes_16k.log 2>&1 || exit $?
cat gpurun_out/dcn2_planes_16k.log
timeout -k 10 400 python bench.py --config c5 --steps 10 --warmup 3 --cpu-seconds 3 --no-f32-compare -o gpurun_out/bench_c5.json > gpurun_out/bench_c5.log 2>&1 || { tail -20 gpurun_out/bench_c5.log; exit 1; }
tail -c 1500 gpurun_out/bench_c5.log
