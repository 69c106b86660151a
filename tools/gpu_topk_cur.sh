#!/bin/bash
# top-k kernel tests, the shard microbench at precision 6 and 0, then the c4 bench
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
run() { echo "+ $*"; "$@"; local rc=$?; if [ $rc -ne 0 ]; then echo "FAILED rc=$rc"; exit $rc; fi; }
run timeout -k 10 600 python -m pytest tests/test_gpu_kernels.py tests/test_gpu_serving.py tests/test_gpu_model.py -x -q -k "topk or retriev or recall or serv or index" -p no:cacheprovider > gpurun_out/topk_tests.log 2>&1
tail -1 gpurun_out/topk_tests.log
PREC=6 run timeout -k 10 300 python tools/microbench_topk.py 12500000 100 64,256,1024
PREC=0 run timeout -k 10 300 python tools/microbench_topk.py 12500000 100 1024
run timeout -k 10 600 python bench.py --config c4 --steps 5 --warmup 2 -o gpurun_out/bench_c4.json
python -c "import json;d=json.load(open('gpurun_out/bench_c4.json'));print(d['ms_per_step'],d['value'],d['roofline']['achieved'],d['roofline']['frac'],d.get('f32_mfma_compare'))"
