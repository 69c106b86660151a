#!/bin/bash
# Round 6: the DP exchange's counts on their own communicator / side stream (no drain at the host
# read). Tests, then the one-GPU rehearsals and the DP sparse microbench.
cd "$(dirname "$0")/.."
tag=${1:-r06e}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 400 --timeout-method thread \
    tests/test_gpu_dp_sparse.py tests/test_gpu_multirank.py tests/test_gpu_inbatch_dedup.py tests/test_gpu_model.py > $out/tests.log 2>&1
rc=$?; tail -3 $out/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/microbench_dp_sparse.py 8 > $out/dp_sparse.log 2>&1 || exit $?
tail -1 $out/dp_sparse.log
for ex in dedupe padded; do
  timeout -k 10 300 python -u bench.py --config c3 --exchange $ex --steps 30 --no-cpu-baseline --no-f32-compare \
      -o $out/c3_exchange_$ex.json > $out/c3_exchange_$ex.log 2>&1 || exit $?
  python3 -c "import json; d=json.load(open('$out/c3_exchange_$ex.json')); print('$ex', d['ms_per_step'], d['config'].get('hipgraph'))"
done
timeout -k 10 300 python -u bench.py --config c3 --eager --extras off --steps 30 --no-cpu-baseline --no-f32-compare \
    -o $out/c3_eager.json > $out/c3_eager.log 2>&1 || exit $?
python3 -c "import json; d=json.load(open('$out/c3_eager.json')); print('eager', d['ms_per_step'])"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $out/tr -o t -- python3 bench.py --config c3 \
    --exchange dedupe --steps 10 --warmup 3 --no-cpu-baseline --no-f32-compare -o $out/c3_exchange_tr.json \
    > $out/c3_exchange_tr.log 2>&1 || exit $?
f=$(find $out/tr -name "*kernel_trace.csv" | head -1)
python3 tools/trace_gaps.py $f > $out/exchange_gaps.txt 2>&1
rm -rf $out/tr
head -30 $out/exchange_gaps.txt
