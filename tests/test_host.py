"""CPU tests: host-side initialisation vs the oracle, topology, and the C-ABI
library's exported symbols (no GPU compute here)."""
import ctypes
import os
import re

import numpy as np
import pytest

from mitgcm_amd import configs
from mitgcm_amd.topology import LatLonTopology
from oracle.harness import gyre_oracle

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _ora(o, name):
    return np.array(o.arr(name))


def test_gyre_grid_bitexact_vs_oracle():
    g, params, state = configs.barotropic_gyre()
    o = gyre_oracle()
    for n in ("dxF", "dyF", "dxG", "dyG", "dxC", "dyC", "dxV", "dyU", "rA", "rAw", "rAs", "recip_dxC",
              "recip_dyC", "recip_dxF", "recip_dyF", "recip_dxV", "recip_dyU", "recip_rA", "recip_rAw",
              "recip_rAs", "fCori", "xC", "yC", "R_low", "Ro_surf", "maskInC", "maskInW", "maskInS",
              "Bo_surf", "recip_Bo", "aW2d", "aS2d", "aC2d", "pW", "pS", "pC"):
        assert np.array_equal(g.f[n], _ora(o, n)), n
    for n in ("hFacC", "hFacW", "hFacS", "recip_hFacW", "recip_hFacS", "maskC", "maskW", "maskS"):
        assert np.array_equal(g.f[n], _ora(o, n).reshape(g.f[n].shape)), n
    for n in ("kSurfC", "kSurfW", "kSurfS", "kLowC"):
        assert np.array_equal(g.i[n], o.iarr(n)), n
    assert g.globalArea == o.get("globalArea")
    assert g.cg2dNorm == o.get("cg2dNorm")
    assert np.array_equal(state["fu"], _ora(o, "fu"))


@pytest.mark.parametrize("nSx,nSy", [(1, 1), (2, 1), (2, 2)])
def test_latlon_exchange_matches_oracle(nSx, nSy):
    from oracle.harness import Oracle
    o = Oracle(8, 6, 2, 2, 3, nSx, nSy)
    rng = np.random.default_rng(1)
    a = rng.standard_normal(o.arr("uVel").shape)
    o.arr("uVel")[:] = a
    o.L.oracle_exch_xyz.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_double), ctypes.c_int]
    o.L.oracle_exch_xyz(o.h, o.arr("uVel").ctypes.data_as(ctypes.POINTER(ctypes.c_double)), 3)
    topo = LatLonTopology(8, 6, 2, 2, nSx, nSy)
    assert np.array_equal(topo.exchange(a), np.array(o.arr("uVel")))


def test_library_exports_every_header_symbol():
    from mitgcm_amd import _lib
    so = os.path.join(ROOT, "mitgcm_amd", "libmitgcm_amd.so")
    if not os.path.exists(so):
        from mitgcm_amd import build
        build.build()
    hdr = open(os.path.join(ROOT, "include", "mitgcm_amd.h")).read()
    declared = set(re.findall(r"\b(mgcm_\w+|\w+_amd_)\s*\(", hdr))
    L = ctypes.CDLL(so)
    for sym in sorted(declared):
        assert hasattr(L, sym), sym
    assert declared == set(_lib.EXPORTS)
