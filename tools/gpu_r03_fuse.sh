#!/bin/bash
# round 3 (session 2): retrieval loss + DCN cross as one autograd node, cached backward seed -- tests, then c3 / c2 timing + trace
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
    -k "dcn or cross or model or multitask or train or c2 or production or golden or deferred or multirank or dedup or inbatch or trainer" \
    > gpurun_out/r03_fuse_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/r03_fuse_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
bash tools/gpu_r03_c3prof.sh > /dev/null || exit $?
grep -E "dcn_cross|Functor|fill|total" gpurun_out/r03_c3_kstats.txt | cut -c1-140
python3 -c "import json;d=json.load(open('gpurun_out/r03_c3_prof_line.json'));print('c3 (profiled)', d['ms_per_step'])"
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --config c3 --steps 50 --warmup 5 --no-cpu-baseline --extras off \
      --no-f32-compare -o gpurun_out/r03_fuse_c3_$i.json > gpurun_out/r03_fuse_c3_$i.log 2>&1 || exit $?
  python3 -c "import json;d=json.load(open('gpurun_out/r03_fuse_c3_$i.json'));print('c3', d['ms_per_step'], d['value'])"
done
timeout -k 10 200 python -u bench.py --config c2 --steps 300 --warmup 20 --no-cpu-baseline --extras off \
    --no-f32-compare -o gpurun_out/r03_fuse_c2.json > gpurun_out/r03_fuse_c2.log 2>&1 || exit $?
python3 -c "import json;d=json.load(open('gpurun_out/r03_fuse_c2.json'));print('c2', d['ms_per_step'], d['value'])"
