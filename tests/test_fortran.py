"""The Fortran side of the boundary (CPU checks; the GPU run is in
test_gpu_parity.py::test_fortran_cg2d_dropin).

* mitgcm_amd/fortran/mods/cg2d.F -- the genmake2 MODS-directory drop-in for
  model/src/cg2d.F -- must compile against the reference's own headers
  (SIZE.h of an experiment, EEPARAMS.h, PARAMS.h, CG2D.h) and export the same
  external symbol (cg2d_) while binding the C-ABI (cg2d_amd_, ini_cg2d_amd_).
  Needs /root/reference (build container only): skipped elsewhere.
* mitgcm_amd/fortran/cg2d_host links against libmitgcm_amd.so.
"""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference"
FC = "/opt/rocm/bin/amdflang"


@pytest.mark.skipif(not (os.path.isdir(REF) and os.path.exists(FC) and shutil.which("cpp")),
                    reason="needs the reference headers and amdflang")
def test_mods_cg2d_compiles_against_reference_headers(tmp_path):
    src = os.path.join(ROOT, "mitgcm_amd", "fortran", "mods", "cg2d.F")
    inc = ["-I" + os.path.join(REF, p) for p in ("verification/tutorial_barotropic_gyre/code", "model/inc",
                                                 "eesupp/inc")]
    pre = subprocess.run(["cpp", "-traditional", "-P", "-DWORDLENGTH=4"] + inc + [src],
                         check=True, capture_output=True, text=True).stdout
    f = tmp_path / "cg2d.f"
    f.write_text(pre.replace(" _d ", "D"))   # genmake2's 64-bit constant rewrite
    obj = tmp_path / "cg2d.o"
    subprocess.run([FC, "-ffixed-form", "-ffixed-line-length=132", "-c", str(f), "-o", str(obj)], check=True)
    syms = subprocess.run(["nm", str(obj)], check=True, capture_output=True, text=True).stdout
    assert " T cg2d_" in syms
    assert " U cg2d_amd_" in syms and " U ini_cg2d_amd_" in syms


@pytest.mark.skipif(not os.path.exists(FC), reason="needs amdflang")
def test_fortran_host_links_library():
    fdir = os.path.join(ROOT, "mitgcm_amd", "fortran")
    subprocess.run(["make", "-s", "-C", fdir], check=True)
    out = subprocess.run(["ldd", os.path.join(fdir, "cg2d_host")], check=True, capture_output=True,
                         text=True).stdout
    assert "libmitgcm_amd.so" in out and "not found" not in out
