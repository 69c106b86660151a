#!/bin/bash
# Round 6: stream-K over XCD key ranges (default build): the in-batch tests, then the C3 kernel
# statistics A/B against the previous order, then FETCH_SIZE / WRITE_SIZE of the pair's passes.
cd "$(dirname "$0")/.."
tag=${1:-r06i}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 400 --timeout-method thread \
    tests/test_gpu_inbatch_dedup.py tests/test_gpu_c3_dedup_at_size.py tests/test_gpu_kernels.py > $out/tests.log 2>&1
rc=$?; tail -n 2 $out/tests.log; [ $rc -eq 0 ] || exit $rc
PROFAB_OUT=$out/ab bash tools/gpu_prof_ab.sh _ablibs/ib_base.so _ablibs/ib_rng.so || exit $?
for lib in ib_base ib_rng; do
  for c in FETCH_SIZE WRITE_SIZE; do
    RECSYS_HIP_LIB=_ablibs/$lib.so timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $c --output-format csv \
        -d $out/pmc_${lib}_$c -o x -- python3 tools/microbench_inbatch_dedup.py 3 > $out/pmc_${lib}_$c.log 2>&1 || exit $?
    f=$(find $out/pmc_${lib}_$c -name '*counter_collection.csv' | head -1)
    echo "== $lib $c" >> $out/pmc.txt
    python3 tools/pmc_summary.py $f inbatch_ >> $out/pmc.txt
    rm -rf $out/pmc_${lib}_$c
  done
done
cut -c1-150 $out/pmc.txt
