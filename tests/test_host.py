"""CPU tests: host-side initialisation vs the oracle, topology, and the C-ABI
library's exported symbols (no GPU compute here)."""
import ctypes
import json
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


def _w2_maps(topo, ldNb=None, ldT=None, mutate=None, want_rc=0, cubed=1):
    """mgcm_exch2_maps (the library's derivation from the W2_EXCH2_TOPOLOGY.h arrays, host
    only) on the arrays of an exch2.py topology (at leading dimensions ldNb, ldT; mutate(a)
    edits them first)."""
    import ctypes
    from mitgcm_amd._lib import lib
    a = topo.w2_arrays(ldNb, ldT)
    if mutate:
        mutate(a)
    IP = lambda x: np.ascontiguousarray(x, dtype=np.int32).ctypes.data_as(ctypes.POINTER(ctypes.c_int))
    keep = {k: np.ascontiguousarray(v, dtype=np.int32) for k, v in a.items() if k.startswith("exch2_")}
    N = topo.nTiles_ * topo.n2
    out = [np.zeros(N, dtype=np.int64) for _ in range(5)]
    LP = lambda x: x.ctypes.data_as(ctypes.POINTER(ctypes.c_long))
    args = [keep[k] for k in ("exch2_tBasex", "exch2_tBasey", "exch2_isNedge", "exch2_isSedge", "exch2_isEedge",
                              "exch2_isWedge", "exch2_nNeighbours", "exch2_neighbourId", "exch2_opposingSend",
                              "exch2_pij", "exch2_oi", "exch2_oj", "exch2_iLo", "exch2_iHi", "exch2_jLo", "exch2_jHi")]
    rc = lib().mgcm_exch2_maps(topo.sNx, topo.sNy, topo.OLx, topo.nTiles_, a["ldNb"], a["ldT"],
                               *[IP(x) for x in args], cubed, *[LP(x) for x in out])
    assert rc == want_rc
    return out


@pytest.mark.parametrize("kind,n,sNx,sNy,OL", [("cube", 32, 32, 32, 4), ("cube", 32, 32, 16, 4), ("cube", 32, 16, 16, 3),
                                               ("llc", 30, 30, 30, 4), ("llc", 90, 90, 90, 4), ("llc", 30, 15, 30, 3)])
def test_exch2_maps_from_w2_arrays(kind, n, sNx, sNy, OL):
    """The library's pkg/exch2 map derivation from the W2_EXCH2_TOPOLOGY.h arrays
    (csrc/exch2_maps.hip, what the Fortran mirror hands it) reproduces, point for point, the
    maps of mitgcm_amd/exch2.py -- the restatement the cube and LLC tests pin to the
    reference's output.txt (solid-body.cs-32x32x1, advect_cs, global_ocean.cs32x15's grid) --
    for the cube at 6, 12 and 24 tiles and the LLC at 13 and 26 tiles."""
    from mitgcm_amd import exch2
    topo = exch2.cube_topology(n, sNx, sNy, OL) if kind == "cube" else exch2.llc_topology(n, sNx, sNy, OL)
    src, u1, v1, u0, v0 = _w2_maps(topo)
    assert np.array_equal(src, topo.src_of_point())
    cu, cv = topo.uv_codes(True)
    assert np.array_equal(u1, cu) and np.array_equal(v1, cv)
    cu, cv = topo.uv_codes(False)
    assert np.array_equal(u0, cu) and np.array_equal(v0, cv)


@pytest.mark.parametrize("out", ["results/output.txt", "results/output.nlfs.txt"])
def test_w2_default_cube_topology_pinned(out):
    """The W2 topology the cs32 harness fills W2_EXCH2_TOPOLOGY.h with (exch2.py's restatement
    of W2_E2SETUP for the default 6-face cube, no data.exch2: w2_set_cs6_facets.F,
    w2_set_map_tiles.F, w2_set_tile2tiles.F) against the reference's own print of it:
    verification/adjustment.cs-32x32x1 lists, per tile, its neighbours' tile ids in W2's order
    for the cube of 32 x 32 faces on 48 tiles of 16 x 8 and on 6 tiles of 32 x 32
    (tests/golden/adjustment.cs-32x32x1/w2_topology.json, make_golden.py)."""
    from mitgcm_amd import exch2
    fx = json.load(open(os.path.join(ROOT, "tests", "golden", "adjustment.cs-32x32x1", "w2_topology.json")))[out]
    topo = exch2.cube_topology(32, fx["sNx"], fx["sNy"], fx["OLx"])
    assert topo.nTiles_ == fx["nSx"] * fx["nSy"] == len(fx["neighbours"])
    w2 = topo.w2_arrays()
    got = [list(w2["exch2_neighbourId"][t, :w2["exch2_nNeighbours"][t]]) for t in range(topo.nTiles_)]
    assert got == fx["neighbours"]


def test_exch2_maps_padded_and_refused():
    """The Fortran mirror passes the W2 arrays at their declared leading dimensions
    (W2_maxNeighbours = 8, W2_maxNbTiles = 2 x the tiles): the maps are those of the unpadded
    arrays.  Inconsistent arrays -- a neighbour id or opposing connection out of range, more
    neighbours than the leading dimension -- are refused (-1), so MGCM_AMD_SET_W2 stops with
    ABNORMAL END instead of setting wrong maps."""
    from mitgcm_amd import exch2
    topo = exch2.cube_topology(32, 32, 16, 4)
    base = _w2_maps(topo)
    padded = _w2_maps(topo, ldNb=8, ldT=2 * topo.nTiles_)
    for x, y in zip(base, padded):
        assert np.array_equal(x, y)

    def bad_id(a):
        a["exch2_neighbourId"][0, 0] = topo.nTiles_ + 1

    def bad_opp(a):
        a["exch2_opposingSend"][1, 0] = 9

    def bad_count(a):
        a["exch2_nNeighbours"][2] = a["ldNb"] + 1
    for m in (bad_id, bad_opp, bad_count):
        _w2_maps(topo, mutate=m, want_rc=-1)


def test_exch2_maps_corners_follow_use_cubed_sphere_exchange():
    """The cube-corner u/v fix-ups sit inside the reference's IF ( useCubedSphereExchange )
    (exch2_uv_3d_rx.template:79): with the flag off the library's maps are those of the two
    EXCH2_RX2_CUBE passes alone -- identical to the flag-on maps everywhere except at the
    corner halo points of tiles with two facet edges, and the scalar map is unchanged."""
    from mitgcm_amd import exch2
    topo = exch2.cube_topology(32, 32, 32, 4)
    on = _w2_maps(topo)
    off = _w2_maps(topo, cubed=0)
    assert np.array_equal(on[0], off[0])
    nx = topo.sNx + 2 * topo.OLx
    corners = set()
    for t in range(topo.nTiles_):
        for i, j in ((0, 0), (1, 0), (0, 1), (0, topo.sNy + 1), (0, topo.sNy + 2), (1, topo.sNy + 2),
                     (topo.sNx + 2, 0), (topo.sNx, 0), (topo.sNx + 1, 0), (topo.sNx + 2, 1),
                     (topo.sNx + 2, topo.sNy + 1), (topo.sNx + 1, topo.sNy + 2), (topo.sNx + 2, topo.sNy),
                     (topo.sNx, topo.sNy + 2)):
            corners.add(t * topo.n2 + (j + topo.OLx - 1) * nx + (i + topo.OLx - 1))
    ndiff = 0
    for a, b in zip(on[1:], off[1:]):
        d = set(np.nonzero(a != b)[0].tolist())
        assert d and d <= corners
        ndiff += len(d)
    assert ndiff > 0
