"""Host driver of the device-resident hot path (the FORWARD_STEP caller).

Model owns one mgcm_model (a tile set in HBM on one GPU): it uploads the
host-initialised grid/masks/operator (grid.py), holds the run-time parameters
(PARAMS.h names), and drives DYNAMICS / SOLVE_FOR_PRESSURE /
MOMENTUM_CORRECTION_STEP / INTEGR_CONTINUITY / DO_FIELDS_BLOCKING_EXCHANGES
through the C-ABI.  There is no CPU path: every call goes to the HIP library.
"""
import ctypes

import numpy as np

from ._lib import check, lib, MgcmError

# fields uploaded from the host-side initialisation
GRID_2D = ("dxF", "dyF", "dxG", "dyG", "dxC", "dyC", "dxV", "dyU", "rA", "rAw", "rAs",
           "recip_dxF", "recip_dyF", "recip_dxC", "recip_dyC", "recip_dxV", "recip_dyU",
           "recip_rA", "recip_rAw", "recip_rAs", "fCori", "Bo_surf", "recip_Bo",
           "aW2d", "aS2d", "aC2d", "pW", "pS", "pC", "maskInC", "tanPhiAtU", "tanPhiAtV",
           "fCoriCos", "recip_Rcol", "rSurfW", "rSurfS", "rLowW", "rLowS", "Ro_surf", "R_low", "maskInW", "maskInS",
           "fCoriG", "recip_rAz", "recip_dxG", "recip_dyG")
GRID_3D = ("hFacC", "hFacW", "hFacS", "recip_hFacC", "recip_hFacW", "recip_hFacS", "maskC", "maskW", "maskS",
           "h0FacC", "h0FacW", "h0FacS")
GRID_1D = ("drF", "drC", "recip_drF", "recip_drC", "rF", "rC")
STATE_1D = ("tRef", "sRef", "pRef4EOS", "phiRefC")
STATE_3D = ("uVel", "vVel", "wVel", "theta", "salt", "gU", "gV", "guNm1", "gvNm1", "gtNm1", "gsNm1", "rhoInSitu",
            "IVDConvCount", "sigmaR", "Kwx", "Kwy", "Kwz", "Kux", "Kvy", "uVelD", "vVelD", "uNM1", "vNM1",
            "totPhiHyd", "alphaRho", "del2u", "del2v", "Kuz", "Kvz", "GM_PsiX", "GM_PsiY")
STATE_2D = ("etaN", "etaH", "fu", "fv", "SST", "lambdaThetaClimRelax", "surfaceForcingT", "surfaceForcingS",
            "Qnet", "EmPmR", "SSS", "lambdaSaltClimRelax", "etaNm1", "rStarFacC", "rStarFacW", "rStarFacS",
            "rStarExpC", "rStarExpW", "rStarExpS", "rStarDhCDt", "rStarDhWDt", "rStarDhSDt", "PmEpR", "dEtaHdt")
# EXTERNAL_FIELDS_LOAD records, in the device's forcRec order
FORCING_ORDER = ("SST", "SSS", "taux", "tauy", "Qnet", "EmPmR")

DEVICE_PARAMS = ("deltaTMom", "deltaTFreeSurf", "deltaTClock", "abEps", "rhoConst", "gBaro", "viscAhD",
                 "viscAhZ", "viscA4D", "viscA4Z", "viscAr", "sideDragFactor", "freeSurfFac", "implicSurfPress",
                 "implicDiv2DFlow", "rkSign", "afFacMom", "vfFacMom", "pfFacMom", "cfFacMom", "foFacMom",
                 "mtFacMom", "momAdvection", "momViscosity", "momForcing", "useCoriolis", "no_slip_sides",
                 "no_slip_bottom", "selectCoriScheme", "momForcingOutAB", "momDissip_In_AB", "implicitViscosity",
                 "cg2dMaxIters", "cg2dUseMinResSol", "nIter0", "vectorInvariantMomentum", "selectVortScheme",
                 "selectKEscheme", "upwindShear")


def _dp(a):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_double))


class Model:
    def __init__(self, grid, params, device=0):
        self.g = grid
        self.params = dict(params)
        L = lib()
        g = grid
        self.h = L.mgcm_create(g.sNx, g.sNy, g.OLx, g.OLy, g.Nr, g.nSx, g.nSy, device)
        if not self.h:
            raise MgcmError("mgcm_create failed: " + L.mgcm_last_error().decode())
        for k, v in self.params.items():
            check(L.mgcm_set_param(self.h, k.encode(), float(v)), "mgcm_set_param(%s)" % k)
        check(L.mgcm_set_param(self.h, b"cg2dNorm", g.cg2dNorm), "cg2dNorm")
        check(L.mgcm_set_param(self.h, b"cg2dTolerance_sq", g.cg2dTolerance_sq), "cg2dTolerance_sq")
        check(L.mgcm_set_param(self.h, b"cg2dNormaliseRHS", float(g.cg2dNormaliseRHS)), "cg2dNormaliseRHS")
        for n in GRID_1D:
            a = np.zeros(g.Nr + 1)
            v = g.f[n]
            a[:len(v)] = v
            self.put(n, a)
        for n in GRID_2D + GRID_3D:
            if n in g.f:        # tanPhiAtU/V exist on spherical grids only
                self.put(n, g.f[n])
        # INI_NLFS_VARS (ini_nlfs_vars.F:79-92): r* factors start at 1
        for n in ("rStarFacC", "rStarFacW", "rStarFacS", "rStarExpC", "rStarExpW", "rStarExpS"):
            self.put(n, np.ones((g.nTiles, g.ny, g.nx)))
        src = np.ascontiguousarray(g.topo.src_of_point(), dtype=np.int64)
        check(L.mgcm_set_halo_map(self.h, src.ctypes.data_as(ctypes.POINTER(ctypes.c_long)), src.size),
              "mgcm_set_halo_map")
        if hasattr(g.topo, "uv_codes"):     # pkg/exch2 topology: C-grid vector maps + cube corners
            topo = g.topo
            LP = lambda a: a.ctypes.data_as(ctypes.POINTER(ctypes.c_long))
            IP = lambda a: a.ctypes.data_as(ctypes.POINTER(ctypes.c_int))
            u1, v1 = (np.ascontiguousarray(x, dtype=np.int64) for x in topo.uv_codes(True))
            u0, v0 = (np.ascontiguousarray(x, dtype=np.int64) for x in topo.uv_codes(False))
            face = np.ascontiguousarray(topo.face[1:], dtype=np.int32)
            edge = np.ascontiguousarray([topo.isN[t] | 2 * topo.isS[t] | 4 * topo.isE[t] | 8 * topo.isW[t]
                                         for t in range(1, topo.nTiles + 1)], dtype=np.int32)
            check(L.mgcm_set_uv_map(self.h, LP(u1), LP(v1), LP(u0), LP(v0), IP(face), IP(edge), u1.size),
                  "mgcm_set_uv_map")

    def init(self):
        check(lib().mgcm_init(self.h), "mgcm_init")

    def close(self):
        if getattr(self, "h", None):
            lib().mgcm_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ---- fields --------------------------------------------------------------
    def _shape(self, name):
        g = self.g
        if name in GRID_1D or name in STATE_1D:
            return (g.Nr + 1,)
        if name in GRID_3D or name in STATE_3D:
            return (g.nTiles, g.Nr, g.ny, g.nx)
        if name == "forcRec":   # 6 forcing fields x the device's record capacity, 2-D each
            n = lib().mgcm_field_count(self.h, b"forcRec")
            return (6, n // (6 * g.nTiles * g.ny * g.nx), g.nTiles, g.ny, g.nx)
        return (g.nTiles, g.ny, g.nx)

    def put_forcing(self, forcing):
        """Upload the periodic forcing records (configs: {name: (nRec, nTiles, ny, nx)})."""
        recs = np.stack([np.asarray(forcing[n], dtype=np.float64) for n in FORCING_ORDER])
        check(lib().mgcm_set_param(self.h, b"nForcRec", float(recs.shape[1])), "nForcRec")
        self.put("forcRec", recs)

    def put(self, name, arr):
        if name == "phiRef":   # set_ref_state.F phiRef(1:2Nr+1): the device keeps phiRef(2k)
            v = np.zeros(self.g.Nr + 1)
            v[:self.g.Nr] = np.asarray(arr)[1:2 * self.g.Nr:2]
            name, arr = "phiRefC", v
        a = np.ascontiguousarray(arr, dtype=np.float64)
        check(lib().mgcm_put(self.h, name.encode(), _dp(a), a.size), "mgcm_put(%s)" % name)

    def get(self, name):
        a = np.zeros(self._shape(name))
        check(lib().mgcm_get(self.h, name.encode(), _dp(a), a.size), "mgcm_get(%s)" % name)
        return a

    # ---- hot path ------------------------------------------------------------
    def prepare(self):
        """Capture the replayed step graph now (outside any timed region)."""
        check(lib().mgcm_prepare(self.h), "mgcm_prepare")

    def forward_step(self, nsteps=1):
        check(lib().mgcm_forward_step(self.h, int(nsteps)), "mgcm_forward_step")

    def thermodynamics(self):
        check(lib().mgcm_thermodynamics(self.h), "mgcm_thermodynamics")

    def dynamics(self):
        check(lib().mgcm_dynamics(self.h), "mgcm_dynamics")

    def solve_for_pressure(self):
        check(lib().mgcm_solve_for_pressure(self.h), "mgcm_solve_for_pressure")

    def my_iter(self):
        """The device-side iteration counter (myIter of the state currently held)."""
        return int(lib().mgcm_get_param(self.h, b"myIter"))

    def sync(self):
        check(lib().mgcm_sync(self.h), "mgcm_sync")

    def solve_stats(self, back=0):
        f, la, rm = ctypes.c_double(), ctypes.c_double(), ctypes.c_double()
        it = ctypes.c_int()
        check(lib().mgcm_solve_stats(self.h, back, ctypes.byref(f), ctypes.byref(la), ctypes.byref(it),
                                     ctypes.byref(rm)), "mgcm_solve_stats")
        return {"cg2d_init_res": f.value, "cg2d_last_res": la.value, "cg2d_iters": it.value,
                "cg2d_rhs_max": rm.value}

    def solve_minres(self, back=0):
        """cg2dUseMinResSol's record of a step's solve: (minResidualSq, nIterMin), -1 when off."""
        r, n = ctypes.c_double(), ctypes.c_int()
        check(lib().mgcm_solve_minres(self.h, back, ctypes.byref(r), ctypes.byref(n)), "mgcm_solve_minres")
        return r.value, n.value

    def solve_history(self, n):
        """numIters, firstResidual, lastResidual of the last n steps (oldest first), one copy."""
        it = np.zeros(n, dtype=np.int32)
        fr = np.zeros(n)
        lr = np.zeros(n)
        check(lib().mgcm_solve_history(self.h, n, it.ctypes.data_as(ctypes.POINTER(ctypes.c_int)), _dp(fr), _dp(lr)),
              "mgcm_solve_history")
        return it, fr, lr

    def cg2d(self, b, x, maxIters, nIterMin=-1):
        b = np.ascontiguousarray(b, dtype=np.float64).copy()
        x = np.ascontiguousarray(x, dtype=np.float64).copy()
        f, mn, la = ctypes.c_double(), ctypes.c_double(), ctypes.c_double()
        it, itm = ctypes.c_int(maxIters), ctypes.c_int(nIterMin)
        check(lib().mgcm_cg2d(self.h, _dp(b), _dp(x), ctypes.byref(f), ctypes.byref(mn), ctypes.byref(la),
                              ctypes.byref(it), ctypes.byref(itm)), "mgcm_cg2d")
        return x, f.value, mn.value, la.value, it.value, itm.value

    def cg2d_sum_plan(self):
        """(plan, NT, PPT, NG): the device CG2D's summation order (mgcm_cg2d_sum_plan)."""
        cap = 1 << 24
        plan = np.zeros(cap, dtype=np.int32)
        nt, ppt, ng = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        check(lib().mgcm_cg2d_sum_plan(self.h, plan.ctypes.data_as(ctypes.POINTER(ctypes.c_int)), cap,
                                       ctypes.byref(nt), ctypes.byref(ppt), ctypes.byref(ng)), "mgcm_cg2d_sum_plan")
        return plan[:nt.value * ppt.value * ng.value].copy(), nt.value, ppt.value, ng.value

    def cg2d_kernel(self):
        """Which CG2D kernel mgcm_init selected: 'mwg' (multi-workgroup), 'bxy' (BX x BY points/thread),
        'blk2' (2x2), 'block', or 'block_ref' (k_cg2d_block summing in the reference's order,
        cg2dRefOrder)."""
        k = lib().mgcm_get_param(self.h, b"cg2dKernel")
        return {5.0: "block_ref", 4.0: "mwg", 3.0: "bxy", 2.0: "blk2"}.get(k, "block")

    def step_layout(self):
        """The launch layout of the last step built (mgcm_get_param 'stepLayout'): which
        fusions of one_step (model.hip) the timed graph and the eager timed pass run."""
        b = int(lib().mgcm_get_param(self.h, b"stepLayout"))
        return {"dyn_thermo_fused": bool(b & 1), "phys_phi_fused": bool(b & 2), "thermo_second_stream": bool(b & 4),
                "late_join": bool(b & 8)}

    def cg2d_fma(self):
        """True when the selected CG2D kernel solves in fused multiply-adds (cg2dUseFMA): the
        device-order oracle must then evaluate the same fma chains (Oracle.set_sum_plan(fma=))."""
        return lib().mgcm_get_param(self.h, b"cg2dFMA") != 0.0

    def cg2d_parts(self):
        """Workgroups (one per CU) the CG2D solve runs on."""
        return int(lib().mgcm_get_param(self.h, b"cg2dParts"))

    def kernel_timing(self, enable):
        lib().mgcm_kernel_timing(self.h, 1 if enable else 0)

    def kernel_ms(self, name):
        n = ctypes.c_int()
        ms = lib().mgcm_kernel_ms(self.h, name.encode(), ctypes.byref(n))
        return ms, n.value


MON_FIELDS = ("eta", "uvel", "vvel", "wvel", "theta", "salt")
MON_STATS = ("max", "min", "mean", "sd", "del2")


def monitor(model):
    """The dynstat block of MONITOR computed on the device (mgcm_monitor): the same keys as
    dynstat(), without downloading the fields."""
    out = np.zeros(len(MON_FIELDS) * len(MON_STATS))
    check(lib().mgcm_monitor(model.h, _dp(out)), "mgcm_monitor")
    return {"dynstat_%s_%s" % (f, s): float(out[i * 5 + j]) for i, f in enumerate(MON_FIELDS)
            for j, s in enumerate(MON_STATS)}


def mon_stats(g, arr, hfac, mask, area, dr):
    """MON_CALC_STATS_RL (pkg/monitor/mon_calc_stats_rl.F) -- host-side monitor of
    downloaded fields; arr/hfac (nTiles, nz, ny, nx), mask/area (nTiles, ny, nx).
    Sums are in the reference's order (tile, k, j, i)."""
    OLx, OLy, sNx, sNy = g.OLx, g.OLy, g.sNx, g.sNy
    nz = arr.shape[1]
    theMin = theMax = 0.0
    noPnts = True
    tNb, tDel2, tVol, tMean = [], [], [], []
    for t in range(arr.shape[0]):
        nb = d2 = vol = mean = 0.0
        for k in range(nz):
            for j in range(1, sNy + 1):
                J = j + OLy - 1
                for i in range(1, sNx + 1):
                    I = i + OLx - 1
                    v = arr[t, k, J, I]
                    msk = mask[t, J, I] * hfac[t, k, J, I]
                    if msk > 0.0:
                        if noPnts:
                            theMin = theMax = v
                            noPnts = False
                        theMin = min(theMin, v)
                        theMax = max(theMax, v)
                        ddx = hfac[t, k, J, I + 1] * hfac[t, k, J, I - 1]
                        if ddx > 0.0:
                            ddx = (arr[t, k, J, I + 1] - v) + (arr[t, k, J, I - 1] - v)
                        ddy = hfac[t, k, J + 1, I] * hfac[t, k, J - 1, I]
                        if ddy > 0.0:
                            ddy = (arr[t, k, J + 1, I] - v) + (arr[t, k, J - 1, I] - v)
                        d2 = d2 + ddx * ddx + ddy * ddy
                        nb = nb + 1.0
                        tv = area[t, J, I] * dr[k] * msk
                        vol = vol + tv
                        mean = mean + tv * v
        tNb.append(nb); tDel2.append(d2); tVol.append(vol); tMean.append(mean)
    gs = lambda xs: sum(xs, 0.0)
    theNb, theDel2, theVol, theMean = gs(tNb), gs(tDel2), gs(tVol), gs(tMean)
    theSD = 0.0
    if theNb > 0.0:
        theDel2 = np.sqrt(theDel2) / theNb
    if theVol > 0.0:
        theMean = theMean / theVol
        sds = []
        for t in range(arr.shape[0]):
            sd = 0.0
            for k in range(nz):
                for j in range(1, sNy + 1):
                    J = j + OLy - 1
                    for i in range(1, sNx + 1):
                        I = i + OLx - 1
                        msk = mask[t, J, I] * hfac[t, k, J, I]
                        if msk > 0.0:
                            tv = area[t, J, I] * dr[k] * msk
                            sd = sd + tv * (arr[t, k, J, I] - theMean) * (arr[t, k, J, I] - theMean)
            sds.append(sd)
        theSD = np.sqrt(gs(sds) / theVol)
    return {"min": theMin, "max": theMax, "mean": theMean, "sd": theSD, "del2": theDel2}


def dynstat(model):
    """dynstat block of MONITOR (pkg/monitor/monitor.F:103-129) for eta, u, v, w, theta."""
    g = model.g
    f = g.f
    out = {}
    eta = model.get("etaN")[:, None]
    # the current hFac (r*: h0Fac*rStarFac, updated every step on the device)
    hC, hW, hS = model.get("hFacC"), model.get("hFacW"), model.get("hFacS")
    for name, arr, hf, mask, area, dr in (
            ("eta", eta, f["maskInC"][:, None], f["maskInC"], f["rA"], f["drF"]),
            ("uvel", model.get("uVel"), hW, f["maskInW"], f["rAw"], f["drF"]),
            ("vvel", model.get("vVel"), hS, f["maskInS"], f["rAs"], f["drF"]),
            ("wvel", model.get("wVel"), f["maskC"], f["maskInC"], f["rA"], f["drC"]),
            ("theta", model.get("theta"), hC, f["maskInC"], f["rA"], f["drF"]),
            ("salt", model.get("salt"), hC, f["maskInC"], f["rA"], f["drF"])):
        st = mon_stats(g, arr, hf, mask, area, dr)
        for k, v in st.items():
            out["dynstat_%s_%s" % (name, k)] = float(v)
    return out
