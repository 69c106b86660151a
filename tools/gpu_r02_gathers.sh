#!/bin/bash
# round 2: gather / multi-gather / dcn2 / xgemm tests, gather A/B, then the c3 and c5 bench lines
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -x -q -m gpu -k "gather or embedding or sparse or dcn2 or multi or planes or xgemm" \
  -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/tests_g.log 2>&1
rc=$?; tail -3 gpurun_out/tests_g.log
if [ $rc -ne 0 ]; then grep -E "^E |FAILED|Error" gpurun_out/tests_g.log | head -40; exit $rc; fi
timeout -k 10 300 python -u tools/microbench_gather2.py > gpurun_out/gather2.log 2>&1 || exit $?
cat gpurun_out/gather2.log
timeout -k 10 400 python bench.py --config c5 --steps 10 --warmup 3 --no-cpu-baseline --no-f32-compare -o gpurun_out/bench_c5.json > gpurun_out/bench_c5.log 2>&1 || { tail -20 gpurun_out/bench_c5.log; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/bench_c5.json')); r=d['roofline']; print('c5', d['ms_per_step'], r['frac'], r['gather']['zipf'])"
timeout -k 10 400 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-f32-compare -o gpurun_out/bench_c3.json > gpurun_out/bench_c3.log 2>&1 || { tail -20 gpurun_out/bench_c3.log; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/bench_c3.json')); r=d['roofline']; print('c3', d['ms_per_step'], r['frac'], r['gather'])"
