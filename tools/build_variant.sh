#!/bin/bash
# An A/B build of librecsys_hip.so: one translation unit recompiled with extra flags, linked with the
# release objects of the others. Usage: tools/build_variant.sh OUT.so unit.hip "-DFOO=1 ..."
set -e
out=$(realpath -m "$1"); unit=$2; flags=$3
cd "$(dirname "$0")/../recommendation-system-maang-nvidia-_amd/csrc"
make -s -j8 >/dev/null
tmp=$(mktemp -d)
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-result -munsafe-fp-atomics \
  -ffp-contract=fast $flags -c "$unit" -o "$tmp/${unit%.hip}.o"
objs=""
for o in build/*.o; do
  if [ "$(basename $o)" = "${unit%.hip}.o" ]; then objs="$objs $tmp/${unit%.hip}.o"; else objs="$objs $o"; fi
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $objs -o "$out"
rm -rf "$tmp"
echo "built $out"
