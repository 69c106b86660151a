#!/bin/bash
# round 4: non-temporal output stores in the skinny GEMM (tools/_exp_skinny_nt.so, built with
# -DSKINNY_NT_STORE) against the default library: c3 lines
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in def nt def nt; do
  if [ $v = nt ]; then export RECSYS_HIP_LIB=$PWD/tools/_exp_skinny_nt.so; else unset RECSYS_HIP_LIB; fi
  timeout -k 10 300 python -u bench.py --config c3 --extras off --no-cpu-baseline --no-f32-compare --steps 40 \
      -o gpurun_out/r04_nt_c3_$v.json > gpurun_out/r04_nt_c3_$v.log 2>&1 || exit $?
  python3 -c "import json; d=json.load(open('gpurun_out/r04_nt_c3_$v.json')); print('c3 $v', d['ms_per_step'], d['value'])"
done
