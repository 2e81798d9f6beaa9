#!/bin/bash
# Build libmitgcm_amd_mw<NT>x<OPT>.so: the library with k_cg2d_mwg compiled for another
# workgroup geometry (NT threads x OPT points per thread); select it with MGCM_LIB=...
set -e
cd "$(dirname "$0")/.."
NT=$1; OPT=$2
B=mitgcm_amd/_build
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -Wno-unused-result -Wno-unused-value \
  -DMGCM_MW_NT=$NT -DMGCM_MW_OPT=$OPT -c mitgcm_amd/csrc/kernels_cg2d_mwg.hip -o $B/kernels_cg2d_mwg_${NT}x${OPT}.o
objs=$(ls $B/*.o | grep -v "kernels_cg2d_mwg" | tr '\n' ' ')
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o mitgcm_amd/libmitgcm_amd_mw${NT}x${OPT}.so $objs $B/kernels_cg2d_mwg_${NT}x${OPT}.o
