#!/bin/bash
# round 4 (after the Dense stack kernels): the whole GPU suite, smoke, the c2 kernel stats (launch
# count per step), the 2-rank gloo bench rehearsal
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread \
    > gpurun_out/r04_z_suite.log 2>&1
rc=$?; echo "suite rc=$rc"; tail -3 gpurun_out/r04_z_suite.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c 'import __graft_entry__ as g; g.smoke()' > gpurun_out/r04_z_smoke.log 2>&1 || exit $?
tail -1 gpurun_out/r04_z_smoke.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_z -o c2 -- python3 bench.py --config c2 \
    --extras off --no-cpu-baseline --no-f32-compare --steps 20 --warmup 3 -o gpurun_out/r04_z_c2_prof.json \
    > gpurun_out/r04_z_prof.log 2>&1 || exit $?
f=$(find gpurun_out/prof_z -name "*results.db" | head -1)
python3 tools/rocpd_stats.py $f gpurun_out/r04_z_c2_kernel_stats.csv 60 > gpurun_out/r04_z_c2_kernel_stats.txt 2>&1
rm -rf gpurun_out/prof_z
head -12 gpurun_out/r04_z_c2_kernel_stats.txt | cut -c1-130
RS_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 4 --warmup 2 --extras off \
    --no-cpu-baseline --no-f32-compare > gpurun_out/r04_z_dp2.log 2>&1 || { tail -20 gpurun_out/r04_z_dp2.log; exit 1; }
tail -1 gpurun_out/r04_z_dp2.log | cut -c1-300
