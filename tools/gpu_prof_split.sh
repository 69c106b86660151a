#!/bin/bash
# PMC (one counter per pass) for the split-precision in-batch pair at B = 65536, then rocprofv3
# kernel stats of the c3 bench (default precision)
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
run() { echo "+ $*"; "$@"; local rc=$?; if [ $rc -ne 0 ]; then echo "FAILED rc=$rc: $*"; exit $rc; fi; }
CTRS="FETCH_SIZE WRITE_SIZE SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE"
for c in $CTRS; do
  run timeout -k 10 300 rocprofv3 --kernel-trace --pmc $c --output-format csv -d gpurun_out/pmc_sp_$c -o x -- \
      python3 tools/microbench_inbatch_prec.py 65536 6
done
for c in $CTRS; do
  f=$(find gpurun_out/pmc_sp_$c -name '*counter_collection.csv' | head -1); echo "== $c"; python tools/pmc_summary.py $f rs::
  t=$(find gpurun_out/pmc_sp_$c -name '*kernel_trace.csv' | head -1); python tools/ktrace_avg.py $t inbatch_
done
run timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c3 -o c3 -- \
    python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-f32-compare -o gpurun_out/prof_bench_c3.json
f=$(find gpurun_out/prof_c3 -name '*kernel_stats.csv' | head -1); python tools/kstats.py $f 25
