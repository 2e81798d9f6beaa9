#!/bin/bash
# The library with kernels_step.hip (DYNAMICS + THERMODYNAMICS) compiled under another AMDGPU
# machine-scheduler strategy (max-ilp | max-memory-clause), into
# mitgcm_amd/_build/diag/libmitgcm_amd_sched_<strategy>.so; select it with MGCM_LIB=...
set -e
cd "$(dirname "$0")/.."
ST=${1:?strategy}
D=mitgcm_amd/_build/diag
mkdir -p $D
F="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -Wno-unused-result -Wno-unused-value"
/opt/rocm/bin/hipcc $F -mllvm -amdgpu-sched-strategy=$ST -c mitgcm_amd/csrc/kernels_step.hip -o $D/kernels_step_$ST.o
objs=""
for o in mitgcm_amd/_build/*.o; do case "$(basename $o)" in kernels_step.o) ;; *) objs="$objs $o";; esac; done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $D/libmitgcm_amd_sched_$ST.so $objs $D/kernels_step_$ST.o
rm $D/kernels_step_$ST.o
echo $D/libmitgcm_amd_sched_$ST.so
