#!/bin/bash
# single-launch slab reduction: GPU tests, then c2 / c5 benches new vs old (tools/_exp_reduce_old.so)
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
run() { echo "+ $*"; "$@"; local rc=$?; if [ $rc -ne 0 ]; then echo "FAILED rc=$rc"; exit $rc; fi; }
run timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/ab_tests.log 2>&1
tail -2 gpurun_out/ab_tests.log
for v in new old new old; do
  if [ $v = old ]; then export RECSYS_HIP_LIB=tools/_exp_reduce_old.so; else unset RECSYS_HIP_LIB; fi
  run timeout -k 10 300 python bench.py --config c2 --steps 100 --warmup 10 --no-cpu-baseline -o gpurun_out/ab_c2_$v.json > /dev/null 2>&1
  python -c "import json;d=json.load(open('gpurun_out/ab_c2_$v.json'));print('$v c2',d['ms_per_step'])"
done
for v in new old; do
  if [ $v = old ]; then export RECSYS_HIP_LIB=tools/_exp_reduce_old.so; else unset RECSYS_HIP_LIB; fi
  run timeout -k 10 300 python bench.py --config c5 --steps 5 --warmup 2 --no-cpu-baseline -o gpurun_out/ab_c5_$v.json > /dev/null 2>&1
  python -c "import json;d=json.load(open('gpurun_out/ab_c5_$v.json'));print('$v c5',d['ms_per_step'])"
done
