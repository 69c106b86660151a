#!/bin/bash
# Round 6: the row read-ahead A/B again in the other order (read-ahead build first), twice.
cd "$(dirname "$0")/.."
tag=${1:-r06n}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
PROFAB_OUT=$out/ab1 bash tools/gpu_prof_ab.sh _ablibs/ib_rpfa.so _ablibs/ib_cpf.so || exit $?
PROFAB_OUT=$out/ab2 bash tools/gpu_prof_ab.sh _ablibs/ib_cpf.so _ablibs/ib_rpfa.so
