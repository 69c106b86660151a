#!/bin/bash
# Round 6, first GPU call: the new C5 at-size parity tests and the id-plan tests on the onesweep
# plan sort, then the C3 bench step under rocprofv3 --kernel-trace --stats for the onesweep build
# (the command that faulted in round 5) and the merge-sort variant (variants/merge.so).
cd "$(dirname "$0")/.."
out=gpurun_out/r06a
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
    tests/test_gpu_c5_at_size.py tests/test_gpu_inbatch_dedup.py tests/test_gpu_c3_dedup_at_size.py \
    > $out/tests.log 2>&1
rc=$?; tail -5 $out/tests.log; [ $rc -eq 0 ] || exit $rc
PROFAB_OUT=$out/profab bash tools/gpu_prof_ab.sh variants/merge.so recommendation-system-maang-nvidia-_amd/librecsys_hip.so
