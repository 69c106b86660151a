#!/bin/bash
# Alternating A/B of librecsys_hip.so variants on the deduplicated in-batch pair at the C3 shape
# (tools/mb_ib_pair.py, 3 rounds). Usage: tools/gpu_ab_pair.sh lib1.so lib2.so ...
set -e
for round in 1 2 3; do
  for lib in "$@"; do
    RECSYS_HIP_LIB=$lib timeout -k 10 120 python tools/mb_ib_pair.py 20 "$round $(basename $lib .so)"
  done
done
