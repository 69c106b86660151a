#!/bin/bash
# experiment builds: tools/_exp_<file>_<name>.so with one source rebuilt under extra flags
#   tools/build_variants.sh gemm "noload:-DRS_GEMM_EXP_NOLOAD" ...
set -e
cd "$(dirname "$0")/../recommendation-system-maang-nvidia-_amd/csrc"
make -j8 >/dev/null
src=$1; shift
objs=""
for o in build/*.o; do [ "$o" != "build/$src.o" ] && objs="$objs $o"; done
for v in "$@"; do
  name=${v%%:*}; flags=${v#*:}
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=fast -munsafe-fp-atomics $flags -c $src.hip -o /tmp/${src}_$name.o
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $objs /tmp/${src}_$name.o -o ../../tools/_exp_${src}_$name.so
  echo built tools/_exp_${src}_$name.so
done
