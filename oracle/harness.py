"""ctypes harness around liboracle.so -- TEST INFRASTRUCTURE.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import
this module.  It drives the CPU restatement (oracle/*.c) of the reference's hot
path and reproduces the reference's %MON statistics for comparison.
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "liboracle.so")
# the same sources built with -fopenmp: tiles over OpenMP threads (Oracle.set(nThreads=...)),
# bit-identical to the sequential build; loaded while USE_OMP is set (bench.py cpu_baseline's
# multi-core figure), the sequential build otherwise
LIB_OMP = os.path.join(HERE, "liboracle_omp.so")
USE_OMP = False
_libs = {}


def build():
    subprocess.check_call(["make", "-s", "-C", HERE])


def lib():
    key = bool(USE_OMP)
    if key not in _libs:
        path = LIB_OMP if key else LIB
        if not os.path.exists(path):
            build()
        L = ctypes.CDLL(path)
        vp, c_int, c_dbl, c_char_p = ctypes.c_void_p, ctypes.c_int, ctypes.c_double, ctypes.c_char_p
        L.oracle_new.restype = vp
        L.oracle_new.argtypes = [c_int] * 7
        L.oracle_free.argtypes = [vp]
        L.oracle_set_param.argtypes = [vp, c_char_p, c_dbl]
        L.oracle_set_param.restype = c_int
        L.oracle_get_param.argtypes = [vp, c_char_p]
        L.oracle_get_param.restype = c_dbl
        L.oracle_array.argtypes = [vp, c_char_p, ctypes.POINTER(ctypes.c_long)]
        L.oracle_array.restype = ctypes.POINTER(c_dbl)
        L.oracle_iarray.argtypes = [vp, c_char_p, ctypes.POINTER(ctypes.c_long)]
        L.oracle_iarray.restype = ctypes.POINTER(c_int)
        for fn in ("oracle_ini_grid", "oracle_ini_cg2d"):
            getattr(L, fn).argtypes = [vp]
            getattr(L, fn).restype = c_int
        L.oracle_ini_depths.argtypes = [vp, ctypes.POINTER(c_dbl)]
        L.oracle_ini_depths.restype = c_int
        for fn in ("oracle_dynamics", "oracle_solve_for_pressure", "oracle_momentum_correction_step",
                   "oracle_integr_continuity", "oracle_forward_step", "oracle_oceanic_phys",
                   "oracle_thermodynamics", "oracle_fields_load", "oracle_ini_nlfs_pickup",
                   "oracle_calc_r_star", "oracle_update_cg2d", "oracle_integr_continuity_init"):
            getattr(L, fn).argtypes = [vp]
        P = ctypes.POINTER(c_dbl)
        L.oracle_cg2d.argtypes = [vp, P, P, P, P, P, ctypes.POINTER(c_int), ctypes.POINTER(c_int)]
        L.oracle_mon_stats.argtypes = [vp, P, c_int, P, c_int, P, P, P, P]
        L.oracle_exch_xy.argtypes = [vp, P]
        LP = ctypes.POINTER(ctypes.c_long)
        IP = ctypes.POINTER(c_int)
        L.oracle_set_exch2.argtypes = [vp, LP, LP, LP, LP, LP, IP, IP]
        L.oracle_set_exch2.restype = c_int
        L.oracle_exch_uv_xyz.argtypes = [vp, P, P, c_int, c_int]
        L.oracle_set_sum_plan.argtypes = [vp, IP, c_int, c_int, c_int]
        L.oracle_set_sum_plan.restype = c_int
        L.oracle_set_cg2d_fma.argtypes = [vp, c_int]
        L.oracle_set_cg2d_fma.restype = c_int
        _libs[key] = L
    return _libs[key]


def _dp(a):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_double))


class Oracle:
    """One oracle model instance (one process, nSx x nSy tiles)."""

    def __init__(self, sNx, sNy, OLx, OLy, Nr, nSx=1, nSy=1):
        self.L = lib()
        self.sNx, self.sNy, self.OLx, self.OLy, self.Nr, self.nSx, self.nSy = sNx, sNy, OLx, OLy, Nr, nSx, nSy
        self.nx, self.ny = sNx + 2 * OLx, sNy + 2 * OLy
        self.h = self.L.oracle_new(sNx, sNy, OLx, OLy, Nr, nSx, nSy)

    def __del__(self):
        if getattr(self, "h", None):
            self.L.oracle_free(self.h)
            self.h = None

    def set(self, **kw):
        for k, v in kw.items():
            if self.L.oracle_set_param(self.h, k.encode(), float(v)) != 0:
                raise KeyError(k)

    def set_sum_plan(self, plan, NT, PPT, NG=1, fma=False):
        """Sum the CG2D dot products in the device's order (mitgcm_amd Model.cg2d_sum_plan());
        fma: the device solves with fused multiply-adds (Model.cg2d_fma()); plan=None restores
        GLOBAL_SUM_TILE_RL's tile order."""
        assert self.L.oracle_set_cg2d_fma(self.h, 1 if fma else 0) == 0
        if plan is None:
            assert self.L.oracle_set_sum_plan(self.h, None, 0, 0, 0) == 0
            return
        p = np.ascontiguousarray(plan, dtype=np.int32)
        assert p.size == NT * PPT * NG
        assert self.L.oracle_set_sum_plan(self.h, p.ctypes.data_as(ctypes.POINTER(ctypes.c_int)), NT, PPT, NG) == 0

    def get(self, name):
        return self.L.oracle_get_param(self.h, name.encode())

    def arr(self, name):
        """Live numpy view of an oracle array, shaped (tiles, [Nr,] ny, nx) for fields."""
        n = ctypes.c_long()
        p = self.L.oracle_array(self.h, name.encode(), ctypes.byref(n))
        if not p:
            raise KeyError(name)
        a = np.ctypeslib.as_array(p, shape=(n.value,))
        nt = self.nSx * self.nSy
        n2 = self.nx * self.ny
        if n.value == nt * n2:
            return a.reshape(nt, self.ny, self.nx)
        if n.value == nt * n2 * self.Nr:
            return a.reshape(nt, self.Nr, self.ny, self.nx)
        return a

    def iarr(self, name):
        n = ctypes.c_long()
        p = self.L.oracle_iarray(self.h, name.encode(), ctypes.byref(n))
        return np.ctypeslib.as_array(p, shape=(n.value,)).reshape(self.nSx * self.nSy, self.ny, self.nx)

    # --- phases ---
    def ini_grid(self):
        assert self.L.oracle_ini_grid(self.h) == 0

    def ini_depths(self, bathy):
        b = np.ascontiguousarray(bathy, dtype=np.float64)
        assert self.L.oracle_ini_depths(self.h, _dp(b)) == 0

    def ini_cg2d(self):
        assert self.L.oracle_ini_cg2d(self.h) == 0

    def forward_step(self):
        self.L.oracle_forward_step(self.h)

    def cg2d(self, b, x, maxIters, nIterMin=-1):
        """CG2D on full halo-inclusive (tiles, ny, nx) arrays; returns (x, first, minSq, last, its, itMin)."""
        b = np.ascontiguousarray(b, dtype=np.float64).copy()
        x = np.ascontiguousarray(x, dtype=np.float64).copy()
        f, mn, la = ctypes.c_double(), ctypes.c_double(), ctypes.c_double()
        it, itm = ctypes.c_int(maxIters), ctypes.c_int(nIterMin)
        self.L.oracle_cg2d(self.h, _dp(b), _dp(x), ctypes.byref(f), ctypes.byref(mn), ctypes.byref(la),
                           ctypes.byref(it), ctypes.byref(itm))
        return x, f.value, mn.value, la.value, it.value, itm.value

    def stats(self, field, nr, hfac, hfac3d, mask, area, dr):
        out = np.zeros(6)
        f = np.ascontiguousarray(field, dtype=np.float64)
        h = np.ascontiguousarray(hfac, dtype=np.float64)
        mk = np.ascontiguousarray(mask, dtype=np.float64)
        ar = np.ascontiguousarray(area, dtype=np.float64)
        d = np.ascontiguousarray(dr, dtype=np.float64)
        self.L.oracle_mon_stats(self.h, _dp(f), nr, _dp(h), int(hfac3d), _dp(mk), _dp(ar), _dp(d), _dp(out))
        return out

    def dynstat(self):
        """The dynstat block of MONITOR (pkg/monitor/monitor.F:103-129) for eta, u, v, w."""
        res = {}
        Nr = self.Nr
        drF = self.arr("drF")[:Nr].copy()
        drC = self.arr("drC")[:Nr].copy()
        mC, mW, mS = self.arr("maskInC"), self.arr("maskInW"), self.arr("maskInS")
        for name, fld, hf, h3, mask, area, dr, nr in (
                ("eta", self.arr("etaN"), mC, 0, mC, self.arr("rA"), drF, 1),
                ("uvel", self.arr("uVel"), self.arr("hFacW"), 1, mW, self.arr("rAw"), drF, Nr),
                ("vvel", self.arr("vVel"), self.arr("hFacS"), 1, mS, self.arr("rAs"), drF, Nr),
                ("wvel", self.arr("wVel"), self.arr("maskC"), 1, mC, self.arr("rA"), drC, Nr),
                ("theta", self.arr("theta"), self.arr("hFacC"), 1, mC, self.arr("rA"), drF, Nr),
                ("salt", self.arr("salt"), self.arr("hFacC"), 1, mC, self.arr("rA"), drF, Nr)):
            st = self.stats(fld, nr, hf, h3, mask, area, dr)
            for key, v in zip(("min", "max", "mean", "sd", "del2"), st[:5]):
                res["dynstat_%s_%s" % (name, key)] = float(v)
        res["cg2d_init_res"] = self.get("firstResidual")
        res["cg2d_iters"] = int(self.get("numIters"))
        res["cg2d_last_res"] = self.get("lastResidual")
        res["cg2d_rhs_max"] = self.get("rhsMax")
        return res


GOLDEN = os.path.join(os.path.dirname(HERE), "tests", "golden")

# host Grid arrays the oracle takes as they are (grid set-up is host-side in the
# product too; the spherical grid is pinned separately by tests/test_grid_sphere.py)
_GRID2 = ("xC", "yC", "xG", "yG", "dxF", "dyF", "dxG", "dyG", "dxC", "dyC", "dxV", "dyU", "rA", "rAw", "rAs",
          "rAz", "recip_dxF", "recip_dyF", "recip_dxG", "recip_dyG", "recip_dxC", "recip_dyC", "recip_dxV",
          "recip_dyU", "recip_rA", "recip_rAw", "recip_rAs", "recip_rAz", "fCori", "fCoriG", "Bo_surf",
          "recip_Bo", "R_low", "Ro_surf", "maskInC", "maskInW", "maskInS", "aW2d", "aS2d", "aC2d", "pW", "pS",
          "pC", "fCoriCos", "tanPhiAtU", "tanPhiAtV")
_GRID3 = ("hFacC", "hFacW", "hFacS", "recip_hFacC", "recip_hFacW", "recip_hFacS", "maskC", "maskW", "maskS")


def oracle_from_config(cfg, **kw):
    """Oracle instance for a mitgcm_amd.configs experiment: parameters and state as
    the config resolves them, grid/masks/CG2D operator copied from the host Grid."""
    g, params, state = cfg(**kw)
    o = Oracle(g.sNx, g.sNy, g.OLx, g.OLy, g.Nr, g.nSx, g.nSy)
    if getattr(g, "usingSphericalPolarGrid", False):
        o.set(usingCartesianGrid=0, usingSphericalPolarGrid=1)
    if getattr(g, "usingCurvilinearGrid", False):
        o.set(usingCartesianGrid=0, usingCurvilinearGrid=1)
    if hasattr(g.topo, "uv_codes"):          # pkg/exch2 topology: install its halo maps
        set_exch2(o, g.topo)
    for k, v in params.items():
        o.set(**{k: v})
    for n in ("drF", "drC", "rF", "rC", "recip_drF", "recip_drC"):
        o.arr(n)[:len(g.f[n])] = g.f[n]
    for n in _GRID2 + _GRID3:
        if n in g.f:
            o.arr(n).reshape(-1)[:] = np.ravel(g.f[n])
    for n in ("kSurfC", "kSurfW", "kSurfS", "kLowC"):
        o.iarr(n)[:] = g.i[n]
    o.set(cg2dNorm=g.cg2dNorm, cg2dTolerance_sq=g.cg2dTolerance_sq, cg2dNormaliseRHS=int(g.cg2dNormaliseRHS),
          globalArea=g.globalArea)
    for n in ("h0FacC", "h0FacW", "h0FacS"):   # INI_MASKS_ETC: h0Fac = hFac at rest
        if n not in state and n in g.f:
            o.arr(n).reshape(-1)[:] = np.ravel(g.f[n])
    for k, v in state.items():
        o.arr(k).reshape(-1)[:len(np.ravel(v))] = np.ravel(v)
    return o, g


def set_exch2(o, topo):
    """Hand the EXCH2 gather maps (mitgcm_amd/exch2.py) and tile face/edge flags to the oracle."""
    c = lambda a: np.ascontiguousarray(a, dtype=np.int64)
    LP = lambda a: a.ctypes.data_as(ctypes.POINTER(ctypes.c_long))
    scal = c(topo.scalar_ids())
    u1, v1 = (c(x) for x in topo.uv_codes(True))
    u0, v0 = (c(x) for x in topo.uv_codes(False))
    face = np.ascontiguousarray(topo.face[1:], dtype=np.int32)
    edge = np.ascontiguousarray([topo.isN[t] | 2 * topo.isS[t] | 4 * topo.isE[t] | 8 * topo.isW[t]
                                 for t in range(1, topo.nTiles + 1)], dtype=np.int32)
    IP = lambda a: a.ctypes.data_as(ctypes.POINTER(ctypes.c_int))
    assert o.L.oracle_set_exch2(o.h, LP(scal), LP(u1), LP(v1), LP(u0), LP(v0), IP(face), IP(edge)) == 0
    o._keep = (scal, u1, v1, u0, v0, face, edge)


def latlon_oracle(**kw):
    """verification/tutorial_global_oce_latlon as the oracle (mitgcm_amd.configs.global_oce_latlon):
    parameters, grid, initial state, and the 12 monthly forcing records EXTERNAL_FIELDS_LOAD
    interpolates."""
    from mitgcm_amd import configs
    g, params, state, forcing = configs.global_oce_latlon(**kw)
    o, _ = oracle_from_config(lambda: (g, params, state))
    names = {"taux": "forcTaux", "tauy": "forcTauy", "Qnet": "forcQnet", "EmPmR": "forcEmPmR", "SST": "forcSST",
             "SSS": "forcSSS"}
    for k, v in forcing.items():
        o.arr(names[k])[:] = np.ravel(v)
    return o, g


def ocean90_oracle(**kw):
    """verification/global_ocean.90x40x15 (BASELINE config 2) as the oracle, restarted from
    its pickups; runs the INITIALISE_VARIA r* sequence (calc_r_star -> update_r_star ->
    update_cg2d -> integr_continuity -> calc_r_star), so dynstat() is the nIter0 monitor."""
    from mitgcm_amd import configs
    g, params, state, forcing = configs.global_ocean_90x40x15(**kw)
    o, _ = oracle_from_config(lambda: (g, params, state))
    names = {"taux": "forcTaux", "tauy": "forcTauy", "Qnet": "forcQnet", "EmPmR": "forcEmPmR", "SST": "forcSST",
             "SSS": "forcSSS"}
    for k, v in forcing.items():
        o.arr(names[k])[:] = np.ravel(v)
    o.L.oracle_ini_nlfs_pickup(o.h)
    return o, g


def cs32x15_oracle(**kw):
    """verification/global_ocean.cs32x15 (cold start, mitgcm_amd.configs.global_ocean_cs32x15)
    as the oracle, with the 12 forcing records and INITIALISE_VARIA's r* sequence."""
    from mitgcm_amd import configs
    g, params, state, forcing = configs.global_ocean_cs32x15(**kw)
    o, _ = oracle_from_config(lambda: (g, params, state))
    names = {"taux": "forcTaux", "tauy": "forcTauy", "Qnet": "forcQnet", "EmPmR": "forcEmPmR", "SST": "forcSST",
             "SSS": "forcSSS"}
    for k, v in forcing.items():
        o.arr(names[k])[:] = np.ravel(v)
    o.L.oracle_ini_nlfs_pickup(o.h)
    return o, g


def read_bin(path, shape, dtype=">f4"):
    return np.fromfile(path, dtype=dtype).astype(np.float64).reshape(shape)


def gyre_oracle():
    """verification/tutorial_barotropic_gyre as the oracle: input/data namelist
    resolved with set_defaults.F / ini_parms.F (values pinned by params.json)."""
    o = Oracle(62, 62, 2, 2, 1)
    o.set(deltaTMom=1200.0, deltaTFreeSurf=1200.0, deltaTClock=1200.0, abEps=0.01,
          viscAhD=400.0, viscAhZ=400.0, f0=1e-4, beta=1e-11, rhoConst=1000.0, gBaro=9.81,
          cg2dTargetResidual=1e-7, cg2dMaxIters=1000, cg2dUseMinResSol=0,
          xgOrigin=-20e3, ygOrigin=-20e3, selectCoriScheme=0, momForcingOutAB=0)
    o.arr("delX")[:] = 20e3
    o.arr("delY")[:] = 20e3
    o.arr("drF")[0] = 5000.0
    o.ini_grid()
    d = os.path.join(GOLDEN, "tutorial_barotropic_gyre")
    o.ini_depths(read_bin(os.path.join(d, "bathy.bin"), (62, 62)))
    o.ini_cg2d()
    fu = read_bin(os.path.join(d, "windx_cosy.bin"), (62, 62))
    F = o.arr("fu")
    F[0, o.OLy:o.OLy + 62, o.OLx:o.OLx + 62] = fu
    o.L.oracle_exch_xy(o.h, _dp(o.arr("fu")))
    o.arr("theta")[:] = 20.0
    o.arr("salt")[:] = 30.0
    return o
