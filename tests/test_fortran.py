"""The Fortran side of the boundary (CPU checks; the GPU runs are tests/test_gpu_fortran.py
and test_gpu_parity.py::test_fortran_cg2d_dropin).

* Every MODS-directory drop-in of mitgcm_amd/fortran/mods -- cg2d.F, dynamics.F,
  thermodynamics.F, do_oceanic_phys.F, solve_for_pressure.F, momentum_correction_step.F,
  integr_continuity.F, update_r_star.F, update_cg2d.F, calc_r_star.F,
  do_fields_blocking_exchanges.F, exch_{xy,xyz,uv_xy,uv_xyz}_rl.F, global_sum_tile.F and
  the mirror set-up mgcm_amd_mirror.F -- must compile against the reference's own headers
  (SIZE.h / CPP_OPTIONS.h of verification/global_ocean.90x40x15, model/inc, eesupp/inc,
  pkg/gmredi, pkg/cd_code: every PARAMS.h / GRID.h / DYNVARS.h / SURFACE.h / FFIELDS.h /
  CG2D.h / GMREDI.h / CD_CODE_VARS.h name it binds must exist), export the reference's
  external symbol and call only entry points libmitgcm_amd.so exports.  Needs
  /root/reference (build container only): skipped elsewhere.
* The Fortran hosts (cg2d_host, fhost) link against libmitgcm_amd.so.
"""
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference"
FC = "/opt/rocm/bin/amdflang"
MODS = os.path.join(ROOT, "mitgcm_amd", "fortran", "mods")
# file -> external symbol of the reference routine it shadows
SHADOWS = {"cg2d.F": "cg2d_", "dynamics.F": "dynamics_", "thermodynamics.F": "thermodynamics_",
           "do_oceanic_phys.F": "do_oceanic_phys_", "solve_for_pressure.F": "solve_for_pressure_",
           "momentum_correction_step.F": "momentum_correction_step_", "integr_continuity.F": "integr_continuity_",
           "update_r_star.F": "update_r_star_", "update_cg2d.F": "update_cg2d_", "calc_r_star.F": "calc_r_star_",
           "do_fields_blocking_exchanges.F": "do_fields_blocking_exchanges_",
           "do_stagger_fields_exchanges.F": "do_stagger_fields_exchanges_", "exch_xy_rl.F": "exch_xy_rl_",
           "exch_xyz_rl.F": "exch_xyz_rl_", "exch_uv_xy_rl.F": "exch_uv_xy_rl_",
           "exch_uv_xyz_rl.F": "exch_uv_xyz_rl_", "global_sum_tile.F": "global_sum_tile_rl_",
           "mgcm_amd_mirror.F": "mgcm_amd_mirror_", "mgcm_amd_exch2.F": "mgcm_amd_exch2_maps_"}
# compiled on the reference's cube-sphere experiment with pkg/exch2 on (its only branch)
EXCH2_ONLY = {"mgcm_amd_exch2.F": "global_ocean.cs32x15"}


def _compile(src, tmp_path, exp, pkgs=("pkg/gmredi", "pkg/cd_code")):
    inc = ["-I" + str(tmp_path)] + ["-I" + os.path.join(REF, p) for p in (
        "verification/%s/code" % exp, "model/inc", "eesupp/inc") + tuple(pkgs)]
    pre = subprocess.run(["cpp", "-traditional", "-P", "-DWORDLENGTH=4"] + inc + [src],
                         check=True, capture_output=True, text=True).stdout
    base = os.path.basename(src)[:-2]
    f = tmp_path / (base + ".f")
    f.write_text(pre.replace(" _d ", "D"))   # genmake2's 64-bit constant rewrite
    obj = tmp_path / (base + ".o")
    subprocess.run([FC, "-ffixed-form", "-ffixed-line-length=132", "-c", str(f), "-o", str(obj)], check=True)
    return subprocess.run(["nm", str(obj)], check=True, capture_output=True, text=True).stdout


@pytest.mark.skipif(not (os.path.isdir(REF) and os.path.exists(FC) and shutil.which("cpp")),
                    reason="needs the reference headers and amdflang")
def test_mods_dropins_compile_against_reference_headers(tmp_path):
    # the package switches genmake2 derives from packages.conf (written here so that the
    # GMREDI and CD-scheme branches of the mirror are compiled too)
    (tmp_path / "PACKAGES_CONFIG.h").write_text("#define ALLOW_GMREDI\n#define ALLOW_CD_CODE\n")
    so = os.path.join(ROOT, "mitgcm_amd", "libmitgcm_amd.so")
    if not os.path.exists(so):
        from mitgcm_amd import build
        build.build()
    exported = set(subprocess.run(["nm", "-D", "--defined-only", so], check=True, capture_output=True,
                                  text=True).stdout.split())
    files = sorted(f for f in os.listdir(MODS) if f.endswith(".F"))
    assert set(files) == set(SHADOWS), files
    defined_here = set(SHADOWS.values()) | {"mgcm_amd_exch_setup_", "mgcm_amd_rparam_", "mgcm_amd_lparam_",
                                            "mgcm_amd_iparam_"}
    x2 = tmp_path / "exch2"
    x2.mkdir()
    (x2 / "PACKAGES_CONFIG.h").write_text("#define ALLOW_EXCH2\n")
    for f in files:
        if f in EXCH2_ONLY:
            syms = _compile(os.path.join(MODS, f), x2, EXCH2_ONLY[f], pkgs=("pkg/exch2",))
        else:
            syms = _compile(os.path.join(MODS, f), tmp_path, "global_ocean.90x40x15")
        assert re.search(r" T %s$" % SHADOWS[f], syms, re.M), (f, syms)
        calls = set(re.findall(r" U (\w+_amd_\w*)$", syms, re.M))
        assert calls, f
        for c in calls - defined_here:
            assert c in exported, (f, c)


@pytest.mark.skipif(not os.path.exists(FC), reason="needs amdflang")
def test_fortran_hosts_link_library():
    fdir = os.path.join(ROOT, "mitgcm_amd", "fortran")
    subprocess.run(["make", "-s", "-C", fdir], check=True)
    for exe in ("cg2d_host", "fhost"):
        out = subprocess.run(["ldd", os.path.join(fdir, exe)], check=True, capture_output=True, text=True).stdout
        assert "libmitgcm_amd.so" in out and "not found" not in out, exe


@pytest.mark.skipif(not (os.path.isdir(REF) and os.path.exists(FC) and shutil.which("cpp")),
                    reason="needs the reference headers and amdflang")
def test_refhost_builds_against_reference_headers():
    """mitgcm_amd/fortran/refhost: the MODS drop-ins + the harness main program + the
    generated COMMON-block fill routines compile against the reference's headers (its own
    SIZE.h and the one-tile layout) and link the library."""
    import sys
    sys.path.insert(0, os.path.join(ROOT, "mitgcm_amd", "fortran"))
    import build_refhost
    params, fields = build_refhost.mirror_calls()
    assert ("R", "monitorFreq") in params and ("I", "nEndIter") in params
    assert {n for n, k in fields if k == 2} == {"fu", "fv", "Qnet", "EmPmR", "SST", "SSS"}
    for exe in build_refhost.build():
        out = subprocess.run(["ldd", exe], check=True, capture_output=True, text=True).stdout
        assert "libmitgcm_amd.so" in out and "not found" not in out, exe
        syms = subprocess.run(["nm", exe], check=True, capture_output=True, text=True).stdout
        for s in ("dynamics_", "mgcm_amd_mirror_", "refhost_param_", "refhost_field_"):
            assert re.search(r" T %s$" % s, syms, re.M), (exe, s)
