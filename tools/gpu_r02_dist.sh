#!/bin/bash
# round 2: the whole GPU suite + smoke(), then the 2-rank data-parallel rehearsal on the one GPU
# (gloo backend; the product path is RCCL) for c2, c3 and c5
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread \
  > gpurun_out/tests_full.log 2>&1
rc=$?; tail -3 gpurun_out/tests_full.log
if [ $rc -ne 0 ]; then grep -E "^E |FAILED|Error" gpurun_out/tests_full.log | head -40; exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" || exit $?
for c in c2 c3 c5; do
  RS_DIST_BACKEND=gloo timeout -k 10 600 python bench.py --gpus 2 --config $c --steps 5 --warmup 2 --no-f32-compare \
    -o gpurun_out/dist2_$c.json > gpurun_out/dist2_$c.log 2>&1 || { tail -30 gpurun_out/dist2_$c.log; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/dist2_$c.json')); print('$c x2', d['n_gpus'], d['ms_per_step'], d['value'])"
done
