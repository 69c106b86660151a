#!/bin/bash
# Per-kernel VGPR / spill / occupancy table of one csrc translation unit (hipcc resource remarks).
# Usage: tools/regs.sh inbatch.hip [name-filter]
cd "$(dirname "$0")/../recommendation-system-maang-nvidia-_amd/csrc" || exit 1
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -munsafe-fp-atomics -ffp-contract=fast $EXTRA \
  -c "$1" -o /tmp/regs_$$.o -Rpass-analysis=kernel-resource-usage 2>&1 |
  awk -v f="${2:-.}" '/Function Name:/ {n=$NF; if (n ~ /^\[/) n=$(NF-1); name=$0; sub(/.*Function Name: /,"",name); sub(/ \[.*/,"",name)}
       /VGPRs: / {v=$0; sub(/.*VGPRs: /,"",v); sub(/ .*/,"",v)}
       /AGPRs: / {a=$0; sub(/.*AGPRs: /,"",a); sub(/ .*/,"",a)}
       /VGPRs Spill: / {s=$0; sub(/.*VGPRs Spill: /,"",s); sub(/ .*/,"",s)}
       /Occupancy/ {o=$0; sub(/.*SIMD\]: /,"",o); sub(/ .*/,"",o)}
       /LDS Size/ {if (name ~ f) printf "%-90s vgpr %4s agpr %3s spill %3s occ %s\n", substr(name,1,90), v, a, s, o}'
rm -f /tmp/regs_$$.o
