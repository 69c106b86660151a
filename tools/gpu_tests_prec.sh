#!/bin/bash
# full GPU tests, then c3 / c5 / c2 benches at the default precision (with the f32 comparison)
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
run() { echo "+ $*"; "$@"; local rc=$?; if [ $rc -ne 0 ]; then echo "FAILED rc=$rc: $*"; exit $rc; fi; }
timeout -k 10 900 python -m pytest tests -q -m gpu -p no:cacheprovider > gpurun_out/tests.log 2>&1
rc=$?; tail -2 gpurun_out/tests.log
if [ $rc -ne 0 ]; then grep -E "^E |FAILED" gpurun_out/tests.log | head -30; exit $rc; fi
run timeout -k 10 600 python bench.py --steps 10 --warmup 3 --no-cpu-baseline -o gpurun_out/bench_c3.json
run timeout -k 10 600 python bench.py --config c5 --steps 5 --warmup 2 --no-cpu-baseline -o gpurun_out/bench_c5.json
run timeout -k 10 300 python bench.py --config c2 --steps 100 --warmup 5 --no-cpu-baseline -o gpurun_out/bench_c2.json
python - <<'PY'
import json
for c in ("c3", "c5", "c2"):
    d = json.load(open(f"gpurun_out/bench_{c}.json"))
    print(c, d["ms_per_step"], d["value"], d["roofline"]["achieved"], d["roofline"]["frac"], d.get("f32_mfma_compare"))
PY
