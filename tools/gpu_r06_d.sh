#!/bin/bash
# Round 6: DP sparse work without sorts (planned local dedupe, merged exchange order) + tests, the
# DP sparse-cost microbench, the one-GPU exchange rehearsals (bench --exchange), and the C3 line.
cd "$(dirname "$0")/.."
tag=${1:-r06d}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 400 --timeout-method thread \
    tests/test_gpu_dp_sparse.py tests/test_gpu_inbatch_dedup.py tests/test_gpu_multirank.py > $out/tests.log 2>&1
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
timeout -k 10 300 python -u bench.py --config c3 --extras off --steps 30 --no-cpu-baseline --no-f32-compare \
    -o $out/c3_graph.json > $out/c3_graph.log 2>&1 || exit $?
python3 -c "
import json
for k in ('eager', 'graph'):
    d = json.load(open('$out/c3_%s.json' % k)); print(k, d['ms_per_step'], d['roofline']['frac'])"
