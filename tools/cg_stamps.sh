#!/bin/bash
# Diagnostic build of the library with per-phase s_memtime stamps in k_cg2d_bxy
# (MGCM_CG_STAMPS), into mitgcm_amd/_build/diag/; run with MGCM_LIB pointing at it.
set -e
cd "$(dirname "$0")/.."
D=mitgcm_amd/_build/diag
mkdir -p $D
F="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -Wno-unused-result -Wno-unused-value"
/opt/rocm/bin/hipcc $F -DMGCM_CG_STAMPS -c mitgcm_amd/csrc/kernels_solve.hip -o $D/kernels_solve.o
objs=""
for o in mitgcm_amd/_build/*.o; do [ "$(basename $o)" = kernels_solve.o ] || objs="$objs $o"; done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $D/libmitgcm_amd_stamps.so $objs $D/kernels_solve.o
echo $D/libmitgcm_amd_stamps.so
