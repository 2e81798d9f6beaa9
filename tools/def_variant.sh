#!/bin/bash
# The library with kernels_step.hip (DYNAMICS + THERMODYNAMICS) compiled with extra flags,
# into mitgcm_amd/_build/diag/libmitgcm_amd_<name>.so; select it with MGCM_LIB=...
#   tools/def_variant.sh <name> "<flags, e.g. -DMGCM_DT_WPE=2>"
set -e
cd "$(dirname "$0")/.."
NAME=${1:?name}; DEFS=${2:-}
D=mitgcm_amd/_build/diag
mkdir -p $D
F="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -Wno-unused-result -Wno-unused-value"
/opt/rocm/bin/hipcc $F $DEFS -c mitgcm_amd/csrc/kernels_step.hip -o $D/kernels_step_$NAME.o
objs=""
for o in mitgcm_amd/_build/*.o; do case "$(basename $o)" in kernels_step.o) ;; *) objs="$objs $o";; esac; done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $D/libmitgcm_amd_$NAME.so $objs $D/kernels_step_$NAME.o
rm $D/kernels_step_$NAME.o
echo $D/libmitgcm_amd_$NAME.so
