#!/bin/bash
# The library with the tracer k-march's waves per SIMD capped at N (MGCM_TRM_WPE) [and the
# implicit solve's at NI], into mitgcm_amd/_build/diag/libmitgcm_amd_wpe<N>[i<NI>].so; select it with MGCM_LIB=...
set -e
cd "$(dirname "$0")/.."
N=${1:?waves}
NI=${2:-}   # optional: the implicit solve's cap too
X=""; TAG=$N; [ -n "$NI" ] && { X="-DMGCM_TRI_WPE=$NI"; TAG=${N}i$NI; }
D=mitgcm_amd/_build/diag
mkdir -p $D
F="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -Wno-unused-result -Wno-unused-value"
/opt/rocm/bin/hipcc $F -DMGCM_TRM_WPE=$N $X -c mitgcm_amd/csrc/kernels_step.hip -o $D/kernels_step_wpe$TAG.o
objs=""
for o in mitgcm_amd/_build/*.o; do case "$(basename $o)" in kernels_step.o) ;; *) objs="$objs $o";; esac; done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $D/libmitgcm_amd_wpe$TAG.so $objs $D/kernels_step_wpe$TAG.o
rm $D/kernels_step_wpe$TAG.o
echo $D/libmitgcm_amd_wpe$TAG.so
