#!/bin/bash
# full GPU tests, the DCN-v2 cross-stack microbench, then the c5 / c3 / c2 benches; stops at the first failure
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
run() { echo "+ $*"; "$@"; local rc=$?; if [ $rc -ne 0 ]; then echo "FAILED rc=$rc: $*"; exit $rc; fi; }
timeout -k 10 900 python -m pytest tests -q -m gpu -p no:cacheprovider > gpurun_out/tests.log 2>&1
rc=$?; tail -4 gpurun_out/tests.log
if [ $rc -ne 0 ]; then grep -E "^E |FAILED" gpurun_out/tests.log | head -30; exit $rc; fi
run timeout -k 10 300 python tools/microbench_dcn2.py 65536 3344 4
run timeout -k 10 300 python tools/microbench_dcn2.py 16384 3344 4
run timeout -k 10 600 python bench.py --config c5 --steps 10 --warmup 2 -o gpurun_out/bench_c5.json
run timeout -k 10 300 python bench.py --config c2 --steps 100 --warmup 5 --no-cpu-baseline -o gpurun_out/bench_c2.json
run timeout -k 10 600 python bench.py --steps 10 --warmup 3 -o gpurun_out/bench_c3.json
cat gpurun_out/bench_c5.json gpurun_out/bench_c2.json gpurun_out/bench_c3.json
