#!/bin/bash
# round-end rehearsal: full GPU tests, smoke(), default bench (with the CPU baseline)
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
run() { echo "+ $*"; "$@"; local rc=$?; if [ $rc -ne 0 ]; then echo "FAILED rc=$rc: $*"; exit $rc; fi; }
timeout -k 10 900 python -m pytest tests -q -m gpu -p no:cacheprovider > gpurun_out/tests.log 2>&1
rc=$?; tail -2 gpurun_out/tests.log
if [ $rc -ne 0 ]; then grep -E "^E |FAILED" gpurun_out/tests.log | head -30; exit $rc; fi
run timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()"
run timeout -k 10 900 python bench.py -o gpurun_out/bench_default.json
