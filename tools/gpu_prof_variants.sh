#!/bin/bash
# rocprofv3 kernel stats of the c3 bench for the current library and each tools/_exp_<FILE>_<v>.so
# (FILE, VARS), filtered by KPAT
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in cur ${VARS}; do
  if [ $v = cur ]; then unset RECSYS_HIP_LIB; else export RECSYS_HIP_LIB=tools/_exp_${FILE}_$v.so; fi
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pv_$v -o c3 -- \
      python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-f32-compare -o gpurun_out/pv_c3_$v.json > /dev/null 2>&1 || exit 1
  echo "== $v $(python -c "import json;print(json.load(open('gpurun_out/pv_c3_$v.json'))['ms_per_step'])")"
  python tools/kstats.py $(find gpurun_out/pv_$v -name "*kernel_stats.csv" | head -1) 60 | grep -E "${KPAT}"
done
