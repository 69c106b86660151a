#!/bin/bash
# experiment builds of the library with top-k variants (tools/_exp_topk_<name>.so)
set -e
cd "$(dirname "$0")/../recommendation-system-maang-nvidia-_amd/csrc"
make -j8 >/dev/null
objs=$(ls build/*.o | grep -v "build/topk.o")
for v in "$@"; do
  name=${v%%:*}; flags=${v#*:}
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=fast $flags -c topk.hip -o /tmp/topk_$name.o
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $objs /tmp/topk_$name.o -o ../../tools/_exp_topk_$name.so
  echo built tools/_exp_topk_$name.so
done
