#!/bin/bash
# Round 6: one C3 step's kernel sequence (rocprofv3 --kernel-trace, release build).
cd "$(dirname "$0")/.."
out=gpurun_out/${1:-r06w}
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $out/trace -o t -- \
    python3 bench.py --config c3 --extras off --steps 5 --warmup 2 --no-cpu-baseline --no-f32-compare \
    -o $out/line.json > $out/prof.log 2>&1 || exit $?
python3 tools/step_sequence.py $out/trace > $out/step_sequence.txt
tail -3 $out/step_sequence.txt
