"""The drop-in boundary's parameter path, on the CPU (no device is touched).

* MGCM_AMD_MIRROR (mitgcm_amd/fortran/mods/mgcm_amd_mirror.F) hands every run-time parameter
  and COMMON-block array to the device under a device name: each name must be the COMMON
  variable's own name, or one of the documented aliases below -- so a binding of the wrong
  variable (e.g. 'diffKhT' bound to diffKhS) is caught here.
* The reference-host harness resolves the run-time parameters from the experiment's own
  namelist files (refhost_parms.F: set_defaults.F, ini_parms.F PARM01-PARM04, data.pkg,
  data.gmredi, set_parms.F / ini_eos.F / gmredi_readparms.F derivations).  `refhost --params`
  writes what the mirror would pass; every value is pinned against the reference's own dump
  of its resolved parameters (verification/<exp>/results/output.txt, parsed into
  tests/golden/<exp>/params.json by tests/golden/make_golden.py) and against the device-side
  configuration of the same experiment (mitgcm_amd/configs.py), for global_ocean.90x40x15
  and global_ocean.cs32x15 (BASELINE configs 2 and 3; the cube-sphere harness is built on
  pkg/exch2, build_refhost.py layout "cs32").
"""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "mitgcm_amd", "fortran", "refhost", "refhost_ref")
PARAM_DIR = os.path.join(ROOT, "tests", "golden", "global_ocean.90x40x15", "input")
sys.path.insert(0, os.path.join(ROOT, "mitgcm_amd", "fortran"))

# device name -> the COMMON variable the mirror passes under it, where they differ:
# uniform vertical profiles by their first level (the mirror refuses non-uniform ones), the
# EOS by the mirror's code, the forcing switch by 0 (the host interpolates the records)
ALIASES = {"viscAr": "viscArNr(1)", "diffKrT": "diffKrNrT(1)", "diffKrS": "diffKrNrS(1)",
           "deltaTtracer": "dTtracerLev(1)", "eosType": "eosCode", "periodicExternalForcing": "zero"}
# the reference's dump prints these profiles under their array names
DUMP_NAMES = {"viscAr": "viscArNr", "diffKrT": "diffKrNrT", "diffKrS": "diffKrNrS", "deltaTtracer": "dTtracerLev"}


def test_mirror_binds_each_name_to_its_own_variable():
    import build_refhost
    calls = [c for c in build_refhost._calls(os.path.join(ROOT, "mitgcm_amd", "fortran", "mods", "mgcm_amd_mirror.F"))
             if c[0] != "#"]
    assert len(calls) > 150
    bad = []
    for c in calls:
        kind, name, arg = c[0], c[1], c[2]
        if kind == "B":
            if arg != name:
                bad.append((name, arg))
        elif arg != name and ALIASES.get(name) != arg:
            bad.append((name, arg))
    assert not bad, bad


def _dump_value(v):
    if isinstance(v, list):
        v = v[0]
    v = v.strip()
    if v in ("T", "F"):
        return 1.0 if v == "T" else 0.0
    if v.startswith("'"):
        return v.strip("'")
    return float(v)


# experiment -> (harness layout, names the reference leaves UNSET, device-config differences):
# global_ocean.cs32x15 (BASELINE config 3, pkg/exch2, staggerTimeStep, no CD scheme: epsAB_CD
# stays unset; the device configuration is its cold start, nIter0 = 0, where the namelist
# restarts from pickup.0000072000)
EXPERIMENTS = {"global_ocean.90x40x15": ("ref", {"selectVortScheme", "temp_EvPrRn"}, ()),
               "global_ocean.cs32x15": ("cs32", {"temp_EvPrRn", "epsAB_CD"}, ("nIter0",))}


@pytest.mark.parametrize("exp", sorted(EXPERIMENTS))
def test_refhost_resolves_the_namelist_as_the_reference(exp, tmp_path):
    layout, unset_ok, cfg_skip = EXPERIMENTS[exp]
    exe = os.path.join(ROOT, "mitgcm_amd", "fortran", "refhost", "refhost_" + layout)
    if not os.path.exists(exe):
        pytest.skip("refhost not built (needs the reference headers)")
    out = tmp_path / "params.txt"
    pdir = os.path.join(ROOT, "tests", "golden", exp, "input")
    r = subprocess.run([exe, "--params", pdir, str(out)], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stdout + r.stderr
    got = {}
    for line in open(out):
        n, v = line.split()
        got[n] = float(v)
    import build_refhost
    names = [n for _, n in build_refhost.mirror_calls()[0]]
    assert set(got) == set(names)
    # nothing left unset but selectVortScheme, which stays UNSET_I without vector-invariant
    # momentum (set_parms.F), and temp_EvPrRn, whose UNSET_RL means "at the local SST"
    # (the reference's dump prints 1.234567E+05 too)
    unset = {n for n, v in got.items() if v in (1.234567e5, 123456789.0)}
    assert unset <= unset_ok, unset
    assert got["vectorInvariantMomentum"] == (1.0 if exp == "global_ocean.cs32x15" else 0.0)
    # pinned against the reference's own resolved-parameter dump
    ref = json.load(open(os.path.join(ROOT, "tests", "golden", exp, "params.json")))
    compared, bad = 0, []
    for n, v in got.items():
        key = DUMP_NAMES.get(n, n)
        if key not in ref or n in ("cg2dNorm", "cg2dTolerance_sq", "cg2dNormaliseRHS"):
            continue
        want = _dump_value(ref[key])
        if n == "eosType":
            want = 1.0 if want.startswith("JMD95") else 0.0 if want == "LINEAR" else -1.0
        compared += 1
        if not (v == want or abs(v - want) <= 1e-15 * abs(want)):   # the dump prints 16 digits
            bad.append((n, v, want))
    assert not bad, bad
    assert compared >= 70, compared
    # and against the device-side configuration of the same experiment (configs.py)
    from mitgcm_amd import configs
    _, params, _, _ = (configs.global_ocean_90x40x15() if layout == "ref" else configs.global_ocean_cs32x15(sNy=16))
    shared = [n for n in got if n in params and n not in ("monitorFreq", "nEndIter") + cfg_skip]
    diff = [(n, got[n], float(params[n])) for n in shared if got[n] != float(params[n])]
    assert len(shared) >= 40 and not diff, (len(shared), diff)


def test_refhost_resolves_the_llc_namelist_as_configured(tmp_path):
    """BASELINE config 5 has no reference experiment: tests/test_gpu_refhost.py writes its
    namelist from configs.llc_synthetic's parameters; refhost (layout "llc30") must resolve it
    back to the same values (the GPU test then pins every mirror parameter against the device
    model's own)."""
    exe = os.path.join(ROOT, "mitgcm_amd", "fortran", "refhost", "refhost_llc30")
    if not os.path.exists(exe):
        pytest.skip("refhost not built (needs the reference headers)")
    from mitgcm_amd import configs
    from test_gpu_refhost import _llc_namelists
    g, params, st = configs.llc_synthetic(n=30)
    pdir = _llc_namelists(str(tmp_path / "input"), params, st["tRef"], st["sRef"], configs.llc_delr(50), g)
    out = tmp_path / "params.txt"
    r = subprocess.run([exe, "--params", pdir, str(out)], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stdout + r.stderr
    got = {ln.split()[0]: float(ln.split()[1]) for ln in open(out)}
    shared = [n for n in got if n in params]
    diff = [(n, got[n], float(params[n])) for n in shared if got[n] != float(params[n])]
    assert len(shared) >= 45 and not diff, (len(shared), diff)
