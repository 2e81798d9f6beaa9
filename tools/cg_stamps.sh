#!/bin/bash
# Diagnostic build of the library with per-phase s_memtime stamps in k_cg2d_bxy and k_cg2d_mwg
# (MGCM_CG_STAMPS), into mitgcm_amd/_build/diag/; run with MGCM_LIB pointing at it.
set -e
cd "$(dirname "$0")/.."
D=mitgcm_amd/_build/diag
mkdir -p $D
F="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -Wno-unused-result -Wno-unused-value"
/opt/rocm/bin/hipcc $F -DMGCM_CG_STAMPS -c mitgcm_amd/csrc/kernels_solve.hip -o $D/kernels_solve.o
/opt/rocm/bin/hipcc $F -DMGCM_CG_STAMPS -c mitgcm_amd/csrc/kernels_cg2d_mwg.hip -o $D/kernels_cg2d_mwg.o
objs=""
for o in mitgcm_amd/_build/*.o; do case "$(basename $o)" in kernels_solve.o|kernels_cg2d_mwg.o) ;; *) objs="$objs $o";; esac; done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $D/libmitgcm_amd_stamps.so $objs $D/kernels_solve.o $D/kernels_cg2d_mwg.o
echo $D/libmitgcm_amd_stamps.so
