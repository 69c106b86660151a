#!/bin/bash
# split top-k: kernel tests, then the c4 bench (precision 6 with the f32 comparison)
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
run() { echo "+ $*"; "$@"; local rc=$?; if [ $rc -ne 0 ]; then echo "FAILED rc=$rc"; exit $rc; fi; }
run timeout -k 10 600 python -m pytest tests/test_gpu_kernels.py -x -q -k "topk" > gpurun_out/topk_tests.log 2>&1
tail -1 gpurun_out/topk_tests.log
run timeout -k 10 600 python bench.py --config c4 --steps 5 --warmup 2 --no-cpu-baseline -o gpurun_out/bench_c4.json
python -c "import json;d=json.load(open('gpurun_out/bench_c4.json'));print(d['ms_per_step'],d['value'],d['roofline']['achieved'],d['roofline']['frac'],d.get('f32_mfma_compare'))"
