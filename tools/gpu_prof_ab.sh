#!/bin/bash
# Kernel statistics of the C3 bench step for two librecsys_hip.so variants and their per-kernel
# difference (us/step). Usage: tools/gpu_prof_ab.sh A.so B.so   (results: gpurun_out/profab/)
cd "$(dirname "$0")/.."
out=${PROFAB_OUT:-gpurun_out/profab}
mkdir -p $out
export TMPDIR=/tmp
for lib in "$1" "$2"; do
  tag=$(basename $lib .so)
  RECSYS_HIP_LIB=$lib timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $out/prof_$tag -o p -- \
      python3 bench.py --config c3 --extras off --steps 20 --warmup 3 --no-cpu-baseline --no-f32-compare \
      -o $out/${tag}_line.json > $out/${tag}_prof.log 2>&1 || exit $?
  f=$(find $out/prof_$tag -name "*results.db" | head -1)
  python3 tools/rocpd_stats.py $f $out/${tag}_kernel_stats.csv 60 > $out/${tag}_kernel_stats.txt 2>&1
  rm -rf $out/prof_$tag
done
python3 tools/kstats_diff.py $out/$(basename $1 .so)_kernel_stats.csv $out/$(basename $2 .so)_kernel_stats.csv 23 30
