#!/bin/bash
# Diagnostic build with per-phase s_memtime stamps in k_mom_vi_m2 (MGCM_VI_STAMPS) into
# mitgcm_amd/_build/diag/libmitgcm_amd_vistamps.so; run with MGCM_LIB pointing at it:
#   MGCM_LIB=mitgcm_amd/_build/diag/libmitgcm_amd_vistamps.so python bench.py ...
set -e
cd "$(dirname "$0")/.."
D=mitgcm_amd/_build/diag
mkdir -p $D
F="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -Wno-unused-result -Wno-unused-value"
/opt/rocm/bin/hipcc $F -DMGCM_VI_STAMPS -c mitgcm_amd/csrc/kernels_step.hip -o $D/kernels_step.o
objs=""
for o in mitgcm_amd/_build/*.o; do case "$(basename $o)" in kernels_step.o) ;; *) objs="$objs $o";; esac; done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $D/libmitgcm_amd_vistamps.so $objs $D/kernels_step.o
echo $D/libmitgcm_amd_vistamps.so
