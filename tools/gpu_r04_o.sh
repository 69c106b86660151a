#!/bin/bash
# round 4: skinny GEMM row blocks per workgroup (RS_SKINNY_BLOCKS) — bitwise check, tower
# microbench and c3 line per setting
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
for nb in 1 2 4; do
  RS_SKINNY_BLOCKS=$nb timeout -k 10 200 python -u tools/skinny_blocks_check.py gpurun_out/skb_$nb.pt || exit $?
done
python3 tools/skinny_blocks_check.py --compare gpurun_out/skb_1.pt gpurun_out/skb_2.pt || exit 1
python3 tools/skinny_blocks_check.py --compare gpurun_out/skb_1.pt gpurun_out/skb_4.pt || exit 1
rm -f gpurun_out/skb_*.pt
for nb in 1 2 4 1 2; do
  echo "== RS_SKINNY_BLOCKS=$nb"
  RS_SKINNY_BLOCKS=$nb timeout -k 10 120 python -u tools/microbench_towers.py 2>&1 | grep -v amdgpu.ids || exit $?
done > gpurun_out/r04_o_towers.log
cat gpurun_out/r04_o_towers.log | grep "total"
for nb in 1 2 1 2; do
  RS_SKINNY_BLOCKS=$nb timeout -k 10 300 python -u bench.py --extras off --no-cpu-baseline --no-f32-compare --steps 40 \
      -o gpurun_out/r04_o_c3_$nb.json > /dev/null 2>&1 || exit $?
  python3 -c "import json; d=json.load(open('gpurun_out/r04_o_c3_$nb.json')); print('blocks $nb', d['ms_per_step'], d['roofline']['frac'])"
done
