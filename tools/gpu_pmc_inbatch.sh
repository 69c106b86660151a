#!/bin/bash
# PMC traffic of the score-storing in-batch pair (one counter per pass, kernel-trace only)
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
run() { echo "+ $*"; "$@"; local rc=$?; if [ $rc -ne 0 ]; then echo "FAILED rc=$rc: $*"; exit $rc; fi; }
for c in FETCH_SIZE WRITE_SIZE; do
  run timeout -k 10 300 rocprofv3 --kernel-trace --pmc $c --output-format csv -d gpurun_out/pmc_ib_$c -o ib -- \
      python3 tools/microbench_inbatch.py 65536 128 stored
  f=$(find gpurun_out/pmc_ib_$c -name '*counter_collection.csv' | head -1); python tools/pmc_summary.py $f inbatch
done
