"""Experiment set-ups of the reference's verification suite, as host-side
configuration (values from the experiment's input/data namelist, resolved with
model/src/set_defaults.F + ini_parms.F; tests pin them against the resolved
parameter dump of the committed results/output.txt).
"""
import os

import math

import numpy as np

from .exch2 import cube_topology
from .grid import Grid
from .model import Model

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")


def read_bin(path, shape, dtype=">f4"):
    """MDS/raw big-endian binary (readBinaryPrec=32 default)."""
    return np.fromfile(path, dtype=dtype).astype(np.float64).reshape(shape)


def barotropic_gyre(nSx=1, nSy=1, data_dir=None, bathy=None, wind=None):
    """verification/tutorial_barotropic_gyre: 62x62x1, code/SIZE.h sNx=sNy=62, OL=2;
    input/data: viscAh=4.E2, f0=1.E-4, beta=1.E-11, rhoConst=1000, gBaro=9.81,
    implicitFreeSurface, deltaT=1200, delX=delY=62*20.E3, x/ygOrigin=-20.E3,
    delR=5000, cg2dTargetResidual=1.E-7, cg2dMaxIters=1000.  Returns (grid, params, state)."""
    d = data_dir or os.path.join(GOLDEN, "tutorial_barotropic_gyre")
    Nx = Ny = 62
    sNx, sNy = Nx // nSx, Ny // nSy
    g = Grid(sNx, sNy, 2, 2, 1, nSx, nSy)
    g.ini_vertical_grid([5000.0])
    g.ini_cartesian_grid(np.full(Nx, 20e3), np.full(Ny, 20e3), -20e3, -20e3)
    g.ini_cori(1e-4, 1e-11, selectCoriMap=1)
    if bathy is None:
        bathy = read_bin(os.path.join(d, "bathy.bin"), (Ny, Nx))
    g.ini_depths_masks(bathy, hFacMin=1.0, hFacMinDr=0.0, gBaro=9.81)
    g.ini_cg2d(1200.0, 1200.0, 1e-7)
    params = dict(deltaTMom=1200.0, deltaTFreeSurf=1200.0, deltaTClock=1200.0, abEps=0.01, rhoConst=1000.0,
                  gBaro=9.81, viscAhD=400.0, viscAhZ=400.0, viscA4D=0.0, viscA4Z=0.0, viscAr=0.0,
                  sideDragFactor=2.0, selectCoriScheme=0, momForcingOutAB=0, momDissip_In_AB=1,
                  cg2dMaxIters=1000, cg2dUseMinResSol=0, nIter0=0, no_slip_sides=1, no_slip_bottom=1)
    if wind is None:
        wind = read_bin(os.path.join(d, "windx_cosy.bin"), (Ny, Nx))
    fu = g.z2()
    inner = g.sl(1, sNx, 1, sNy)
    for t in range(g.nTiles):
        bi, bj = t % nSx, t // nSx
        fu[t][inner] = wind[bj * sNy:(bj + 1) * sNy, bi * sNx:(bi + 1) * sNx]
    state = {"fu": g.exch(fu), "fv": g.z2(), "theta": np.full((g.nTiles, 1, g.ny, g.nx), 20.0),
             "salt": np.full((g.nTiles, 1, g.ny, g.nx), 30.0)}
    return g, params, state


BAROCLINIC_DELR = [50., 60., 70., 80., 90., 100., 110., 120., 130., 140., 150., 160., 170., 180., 190.]
BAROCLINIC_TREF = [30., 27., 24., 21., 18., 15., 13., 11., 9., 7., 6., 5., 4., 3., 2.]


def advect_xy_ab3_c4(nSx=1, nSy=2):
    """verification/advect_xy with input.ab3_c4 (results/output.ab3_c4.txt): the same box and
    flow as advect_xy, theta AND salt advected with the centred 4th-order scheme
    (tempAdvScheme = saltAdvScheme = 4, not multi-dimensional: gad_c4_adv_x/y.F inside
    GAD_CALC_RHS), the tendencies stepped with ADAMS_BASHFORTH3 (code/CPP_OPTIONS.h defines
    ALLOW_ADAMSBASHFORTH_3; alph_AB = 0.5, beta_AB = 0.281105), deltaT = 2750, theta a Gaussian
    bump exp(-(rD/20 km)^2/2) (code/ini_theta.F), salt the +1 psu disc (code/ini_salt.F)."""
    g, params, state = advect_xy(nSx, nSy)
    g.ini_cg2d(2750.0, 2750.0, 1e-13)
    params.update(deltaTMom=2750.0, deltaTFreeSurf=2750.0, deltaTClock=2750.0, deltaTtracer=2750.0, abEps=0.01,
                  tempStepping=1, tempAdvection=1, tempForcing=0, tempAdvScheme=4, tempVertAdvScheme=4,
                  saltAdvScheme=4, saltVertAdvScheme=4, diffKhT=0.0, diffKrT=0.0, useAB3=1, alph_AB=0.5,
                  beta_AB=0.281105)
    rC = g.f["rC"][0]
    theta = np.full((g.nTiles, 1, g.ny, g.nx), 20.0)   # tRef in the halo before the exchange
    for t in range(g.nTiles):
        for J in range(g.OLy, g.OLy + g.sNy):
            for I in range(g.OLx, g.OLx + g.sNx):
                x, y = g.f["xC"][t, J, I], g.f["yC"][t, J, I]
                rD = math.sqrt((x - 40.0e3) ** 2 + (y - 40.0e3) ** 2 + (rC + 50.0e3) ** 2)
                theta[t, 0, J, I] = math.exp(-0.5 * (rD / 20.0e3) ** 2)
    state["theta"] = g.exch(theta)
    return g, params, state


def baroclinic_gyre(nSx=2, nSy=2, data_dir=None, tempAdvScheme=2):
    """verification/tutorial_baroclinic_gyre: 62x62x15 on a 1-degree spherical-polar
    grid, code/SIZE.h sNx=sNy=31, OL=2, nSx=nSy=2; input/data: viscAh=5000,
    viscAr=1e-2, no_slip_bottom=F, diffKhT=1000, diffKrT=1e-5, ivdc_kappa=1,
    implicitDiffusion, LINEAR EOS tAlpha=2e-4 sBeta=0, rhoNil=999.8, exactConserv,
    saltStepping=F, deltaT=1200, tauThetaClimRelax=2592000 (SST_relax.bin),
    xgOrigin=-1, ygOrigin=14, delR as below.  Resolved parameters are pinned
    against the output.txt dump (tests/test_oracle_3d.py)."""
    d = data_dir or os.path.join(GOLDEN, "tutorial_baroclinic_gyre")
    Nx = Ny = 62
    Nr = 15
    sNx, sNy = Nx // nSx, Ny // nSy
    g = Grid(sNx, sNy, 2, 2, Nr, nSx, nSy)
    g.ini_vertical_grid(BAROCLINIC_DELR)
    g.ini_spherical_polar_grid(np.full(Nx, 1.0), np.full(Ny, 1.0), -1.0, 14.0)
    g.ini_cori(selectCoriMap=2)
    bathy = read_bin(os.path.join(d, "bathy.bin"), (Ny, Nx))
    g.ini_depths_masks(bathy, hFacMin=1.0, hFacMinDr=0.0, gBaro=9.81)
    g.ini_cg2d(1200.0, 1200.0, 1e-7)
    tRef = np.array(BAROCLINIC_TREF)
    params = dict(deltaTMom=1200.0, deltaTFreeSurf=1200.0, deltaTClock=1200.0, deltaTtracer=1200.0, abEps=0.01,
                  rhoConst=999.8, rhoNil=999.8, gravity=9.81, gBaro=9.81, viscAhD=5000.0, viscAhZ=5000.0,
                  viscA4D=0.0, viscA4Z=0.0, viscAr=1e-2, sideDragFactor=2.0, selectCoriScheme=0,
                  momForcingOutAB=0, momDissip_In_AB=1, cg2dMaxIters=1000, cg2dUseMinResSol=0, nIter0=0,
                  no_slip_sides=1, no_slip_bottom=0, exactConserv=1, tempStepping=1, tempAdvection=1,
                  tempForcing=1, tempAdvScheme=tempAdvScheme, tempVertAdvScheme=tempAdvScheme, diffKhT=1000.0,
                  diffKrT=1e-5, ivdc_kappa=1.0, implicitDiffusion=1, tAlpha=2e-4, sBeta=0.0,
                  usingSphericalPolarGrid=1, selectMetricTerms=1, rSphere=g.rSphere, integr_GeoPot=2)
    wind = read_bin(os.path.join(d, "windx_cosy.bin"), (Ny, Nx))
    sst = read_bin(os.path.join(d, "SST_relax.bin"), (Ny, Nx))
    fu, SST = g.z2(), g.z2()
    inner = g.sl(1, sNx, 1, sNy)
    for t in range(g.nTiles):
        bi, bj = t % nSx, t // nSx
        fu[t][inner] = wind[bj * sNy:(bj + 1) * sNy, bi * sNx:(bi + 1) * sNx]
        SST[t][inner] = sst[bj * sNy:(bj + 1) * sNy, bi * sNx:(bi + 1) * sNx]
    theta = np.broadcast_to(tRef[None, :, None, None], (g.nTiles, Nr, g.ny, g.nx)).copy()
    lam = np.full((g.nTiles, g.ny, g.nx), 1.0 / 2592000.0)      # ini_forcing.F:46-51
    state = {"fu": g.exch(fu), "fv": g.z2(), "theta": theta, "salt": np.full_like(theta, 30.0),
             "SST": g.exch(SST), "lambdaThetaClimRelax": lam, "tRef": tRef, "sRef": np.full(Nr, 30.0)}
    return g, params, state


def advect_xy(nSx=1, nSy=2):
    """verification/advect_xy: 20x20x1 doubly-periodic cartesian box (10 km cells,
    code/SIZE.h sNx=20, sNy=10, OL=3, nSy=2), momStepping=F, uniform u = v = 1 m/s
    (code/ini_vel.F), a salt disc of +1 psu (code/ini_salt.F), saltAdvScheme=33
    (DST3 flux-limited, multi-dimensional), deltaT=2500.  Only salt is stepped here
    (theta uses scheme 80 in the reference and does not feed back)."""
    Nx = Ny = 20
    sNx, sNy = Nx // nSx, Ny // nSy
    g = Grid(sNx, sNy, 3, 3, 1, nSx, nSy)
    g.ini_vertical_grid([10.0e3])
    g.ini_cartesian_grid(np.full(Nx, 10.0e3), np.full(Ny, 10.0e3), 0.0, 0.0)
    g.ini_cori(0.0, 0.0, selectCoriMap=1)
    g.ini_depths_masks(np.full((Ny, Nx), g.f["rF"][1]), hFacMin=1.0, hFacMinDr=0.0, gBaro=9.81)
    g.ini_cg2d(2500.0, 2500.0, 1e-13)
    params = dict(deltaTMom=2500.0, deltaTFreeSurf=2500.0, deltaTClock=2500.0, deltaTtracer=2500.0, abEps=0.1,
                  rhoConst=999.8, gravity=9.81, gBaro=9.81, momStepping=0, tempStepping=0, saltStepping=1,
                  saltAdvScheme=33, saltVertAdvScheme=33, multiDimAdvection=1, diffKhS=0.0, diffKrS=0.0,
                  implicitDiffusion=0, ivdc_kappa=0.0, exactConserv=0, saltForcing=0, cg2dMaxIters=100)
    u = np.ones((g.nTiles, 1, g.ny, g.nx)) * g.f["maskW"]
    v = np.ones((g.nTiles, 1, g.ny, g.nx)) * g.f["maskS"]
    salt = np.full((g.nTiles, 1, g.ny, g.nx), 35.0)
    rC = g.f["rC"][0]
    from math import sqrt
    for t in range(g.nTiles):
        for J in range(g.ny):
            for I in range(g.nx):
                x, y = g.f["xC"][t, J, I], g.f["yC"][t, J, I]
                rD = sqrt((x - 40.0e3) ** 2 + (y - 40.0e3) ** 2 + (rC + 50.0e3) ** 2)
                if rD <= 60.0e3:
                    salt[t, 0, J, I] = 35.0 + 1.0
    state = {"uVel": u, "vVel": v, "salt": g.exch(salt), "theta": np.full_like(salt, 20.0),
             "tRef": np.array([20.0]), "sRef": np.array([35.0])}
    return g, params, state


def make_model(cfg, device=0, **kw):
    out = cfg(**kw)
    g, params, state = out[:3]
    m = Model(g, params, device=device)
    for k, v in state.items():
        m.put(k, v)
    if len(out) > 3:
        m.put_forcing(out[3])
    m.init()
    return m


LATLON_DELR = [50., 70., 100., 140., 190., 240., 290., 340., 390., 440., 490., 540., 590., 640., 690.]
# monthly forcing files (12 records each, fp32 big-endian, 90x40) -> FFIELDS.h names
LATLON_FORCING = {"taux": "trenberth_taux.bin", "tauy": "trenberth_tauy.bin", "Qnet": "ncep_qnet.bin",
                  "EmPmR": "ncep_emp.bin", "SST": "lev_sst.bin", "SSS": "lev_sss.bin"}


def _to_tiles(g, glob):
    """Global (..., Ny, Nx) field -> tile layout (..., nTiles, ny, nx), halos exchanged."""
    lead = glob.shape[:-2]
    out = np.zeros(lead + (g.nTiles, g.ny, g.nx))
    inner = g.sl(1, g.sNx, 1, g.sNy)
    for t in range(g.nTiles):
        bi, bj = t % g.nSx, t // g.nSx
        out[(Ellipsis, t) + inner] = glob[..., bj * g.sNy:(bj + 1) * g.sNy, bi * g.sNx:(bi + 1) * g.sNx]
    if out.ndim == 3:
        return g.exch(out)
    flat = out.reshape((-1,) + out.shape[-3:])
    return np.stack([g.exch(f) for f in flat]).reshape(out.shape)


def global_oce_latlon(nSx=2, nSy=1, OL=2, data_dir=None):
    """verification/tutorial_global_oce_latlon: 90x40x15 on a 4-degree spherical-polar
    grid (ygOrigin=-80), code/SIZE.h sNx=45, sNy=40, OL=2, nSx=2; input/data:
    viscAh=5e5, viscAr=1e-3, diffKrT=diffKrS=3e-5, JMD95Z, ivdc_kappa=100,
    implicitDiffusion, allowFreezing, exactConserv, useRealFreshWaterFlux, useCDscheme
    (tauCD=321428), hFacMin=0.05, hFacMinDr=50, deltaTmom=1800, deltaTtracer=
    deltaTClock=deltaTfreesurf=86400, abEps=0.1, monthly periodic forcing (period
    2592000, cycle 31104000), SST/SSS relaxation (5184000 s, 15552000 s), GM-Redi
    (data.gmredi).  Cold start from record 1 of lev_t/lev_s (INI_THETA / INI_SALT:
    masked, theta >= -1.9).  Returns (grid, params, state, forcing) with forcing[name]
    of shape (12, nTiles, ny, nx) (EXTERNAL_FIELDS_LOAD records; EmPmR already in
    kg/m2/s, x rhoConstFresh)."""
    d = data_dir or os.path.join(GOLDEN, "tutorial_global_oce_latlon")
    Nx, Ny, Nr = 90, 40, 15
    g = Grid(Nx // nSx, Ny // nSy, OL, OL, Nr, nSx, nSy)
    g.ini_vertical_grid(LATLON_DELR)
    g.ini_spherical_polar_grid(np.full(Nx, 4.0), np.full(Ny, 4.0), 0.0, -80.0)
    g.ini_cori(selectCoriMap=2)
    bathy = read_bin(os.path.join(d, "bathymetry.bin"), (Ny, Nx))
    g.ini_depths_masks(bathy, hFacMin=0.05, hFacMinDr=50.0, gBaro=9.81)
    g.ini_cg2d(1800.0, 86400.0, 1e-13)
    rhoConstFresh = 1000.0
    forcing = {}
    for name, fn in LATLON_FORCING.items():
        rec = read_bin(os.path.join(d, fn), (12, Ny, Nx))
        if name == "EmPmR":
            rec = rec * rhoConstFresh
        forcing[name] = _to_tiles(g, rec)
    mC = g.f["maskC"]
    theta = _to_tiles(g, read_bin(os.path.join(d, "lev_t.bin"), (Nr, Ny, Nx)))
    theta = np.moveaxis(theta, 0, 1).copy()            # (nTiles, Nr, ny, nx)
    theta[mC == 0.0] = 0.0
    theta = np.where(theta < -1.9, -1.9, theta)         # ini_theta.F: checkIniTemp .AND. allowFreezing
    salt = np.moveaxis(_to_tiles(g, read_bin(os.path.join(d, "lev_s.bin"), (Nr, Ny, Nx))), 0, 1).copy()
    salt[mC == 0.0] = 0.0
    params = dict(deltaTMom=1800.0, deltaTFreeSurf=86400.0, deltaTClock=86400.0, deltaTtracer=86400.0,
                  abEps=0.1, rhoConst=1035.0, rhoConstFresh=rhoConstFresh, gravity=9.81,
                  gBaro=9.81, viscAhD=5e5, viscAhZ=5e5, viscA4D=0.0, viscA4Z=0.0, viscAr=1e-3,
                  sideDragFactor=2.0, selectCoriScheme=0, momForcingOutAB=0, momDissip_In_AB=1,
                  cg2dMaxIters=500, cg2dUseMinResSol=0, nIter0=0, no_slip_sides=1, no_slip_bottom=1,
                  exactConserv=1, tempStepping=1, tempAdvection=1, tempForcing=1, tempAdvScheme=2,
                  tempVertAdvScheme=2, saltStepping=1, saltAdvection=1, saltForcing=1, saltAdvScheme=2,
                  saltVertAdvScheme=2, diffKhT=0.0, diffKrT=3e-5, diffKhS=0.0, diffKrS=3e-5,
                  ivdc_kappa=100.0, implicitDiffusion=1, usingSphericalPolarGrid=1, selectMetricTerms=1,
                  rSphere=g.rSphere, integr_GeoPot=2, eosType=1, allowFreezing=1,
                  useRealFreshWaterFlux=1, useCDscheme=1, tauCD=321428.0, rCD=1.0 - 1800.0 / 321428.0,
                  epsAB_CD=0.1, HeatCapacity_Cp=3994.0, convertFW2Salt=-1.0, temp_EvPrRn=123456.7,
                  salt_EvPrRn=0.0, periodicExternalForcing=1,
                  externForcingPeriod=2592000.0, externForcingCycle=31104000.0, useGMRedi=1,
                  GM_background_K=1e3, GM_isopycK=1e3, GM_skewflx=1.0, GM_maxSlope=1e-2, GM_Kmin_horiz=50.0)
    # set_ref_state.F:92-97: pRef4EOS(k) = top_Pres + rhoConst*(rC(k)-rF(1))*gravity*gravitySign
    pRef = np.array([0.0 + 1035.0 * (g.f["rC"][k] - g.f["rF"][0]) * 9.81 * -1.0 for k in range(Nr)])
    lamT = np.full((g.nTiles, g.ny, g.nx), 1.0 / 5184000.0)    # ini_forcing.F
    lamS = np.full((g.nTiles, g.ny, g.nx), 1.0 / 15552000.0)
    state = {"theta": theta, "salt": salt, "tRef": np.full(Nr, 20.0), "sRef": np.full(Nr, 35.0),
             "pRef4EOS": pRef,
             "lambdaThetaClimRelax": lamT, "lambdaSaltClimRelax": lamS,
             # INI_FORCING: record 1 of every file (the step-0 monitor shows these)
             "fu": forcing["taux"][0], "fv": forcing["tauy"][0], "Qnet": forcing["Qnet"][0],
             "EmPmR": forcing["EmPmR"][0], "SST": forcing["SST"][0], "SSS": forcing["SSS"][0]}
    return g, params, state, forcing


PICKUP_FIELDS = ("uVel", "vVel", "theta", "salt", "guNm1", "gvNm1", "gtNm1", "gsNm1", "totPhiHyd")
PICKUP_2D = ("etaN", "dEtaHdt", "etaH")
PICKUP_CD = ("uVelD", "vVelD", "uNM1", "vNM1")


def read_pickup(g, path, Nx, Ny):
    """READ_PICKUP (model/src/read_pickup.F:170-300): the 12-field MDS pickup (fp64,
    big-endian, global Nx x Ny records) -> tile layout with halos exchanged, as
    READ_PICKUP's EXCH calls leave them (read_pickup.F:545-575)."""
    Nr = g.Nr
    if not os.path.exists(path) and os.path.exists(path + ".data"):
        path = path + ".data"   # written by pickup.write_pickup (MDS name); the fixture has none
    raw = np.fromfile(path, dtype=">f8").astype(np.float64)
    nrec = len(PICKUP_FIELDS) * Nr + len(PICKUP_2D)
    if raw.size != nrec * Nx * Ny:
        raise ValueError("%s: %d values, expected %d records of %dx%d" % (path, raw.size, nrec, Nx, Ny))
    raw = raw.reshape(nrec, Ny, Nx)
    out = {}
    for n, name in enumerate(PICKUP_FIELDS):
        out[name] = np.moveaxis(_to_tiles(g, raw[n * Nr:(n + 1) * Nr]), 0, 1).copy()
    base = len(PICKUP_FIELDS) * Nr
    for n, name in enumerate(PICKUP_2D):
        out[name] = _to_tiles(g, raw[base + n])
    return out


def read_pickup_cd(g, path, Nx, Ny):
    """CD_CODE_READ_PICKUP (pkg/cd_code/cd_code_read_pickup.F:53-69): uVelD, vVelD,
    uNM1, vNM1 (Nr records each) and etaNm1 (record 4*Nr+1)."""
    Nr = g.Nr
    if not os.path.exists(path) and os.path.exists(path + ".data"):
        path = path + ".data"
    raw = np.fromfile(path, dtype=">f8").astype(np.float64).reshape(-1, Ny, Nx)
    out = {}
    for n, name in enumerate(PICKUP_CD):
        out[name] = np.moveaxis(_to_tiles(g, raw[n * Nr:(n + 1) * Nr]), 0, 1).copy()
    out["etaNm1"] = _to_tiles(g, raw[4 * Nr])
    return out


def global_ocean_90x40x15(nSx=1, nSy=1, OL=3, data_dir=None, pickup_dir=None, nIter0=36000, params_over=None):
    """verification/global_ocean.90x40x15 (BASELINE config 2): the lat-lon grid, bathymetry
    and monthly forcing of tutorial_global_oce_latlon (input/prepare_run links them),
    restarted from pickup.0000036000 + pickup_cd.0000036000.  input/data differences:
    viscA4=1e14 (biharmonic, needs OL >= 3), gravity=9.81, eosType='JMD95P'
    (selectP_inEOS_Zc=2: pressure from totPhiHyd), ivdc_kappa=10, select_rStar=2,
    nonlinFreeSurf=4 (r* coordinate, UPDATE_CG2D every step), hFacInf=0.2, hFacSup=2,
    quasiHydrostatic + useNHMTerms (+ use3dCoriolis default), doResetHFactors,
    nIter0=36000 (another nIter0 restarts from pickup(_cd).<nIter0> in pickup_dir, e.g. one
    pickup.write_pickup wrote).  Returns (grid, params, state, forcing); state includes the
    pickups."""
    d = data_dir or os.path.join(GOLDEN, "tutorial_global_oce_latlon")
    pd = pickup_dir or os.path.join(GOLDEN, "global_ocean.90x40x15")
    g, params, state, forcing = global_oce_latlon(nSx=nSx, nSy=nSy, OL=OL, data_dir=d)
    Nx, Ny, Nr = 90, 40, 15
    params.update(viscA4D=1e14, viscA4Z=1e14, ivdc_kappa=10.0, nIter0=nIter0, myIter=nIter0,
                  myTime=nIter0 * 86400.0, selectP_inEOS_Zc=2, storePhiHyd4Phys=1, nonlinFreeSurf=4,
                  select_rStar=2, hFacInf=0.2, hFacSup=2.0, quasiHydrostatic=1, useNHMTerms=1,
                  select3dCoriScheme=1, cg2dPreCondFreq=1)
    # set_ref_state.F:85-97 (top_Pres = 0, gravityFile = ' ')
    rC, rF = g.f["rC"], g.f["rF"]
    phiRef = np.zeros(2 * Nr + 1)
    for k in range(Nr):
        phiRef[2 * k + 1] = phiRef[0] + (rC[k] - rF[0]) * 9.81 * -1.0
        phiRef[2 * k + 2] = phiRef[0] + (rF[k + 1] - rF[0]) * 9.81 * -1.0
    state = {k: v for k, v in state.items() if k not in ("theta", "salt")}
    state["phiRef"] = phiRef
    state.update(read_pickup(g, os.path.join(pd, "pickup.%010d" % nIter0), Nx, Ny))
    state.update(read_pickup_cd(g, os.path.join(pd, "pickup_cd.%010d" % nIter0), Nx, Ny))
    for n in ("h0FacC", "h0FacW", "h0FacS", "recip_Rcol", "rLowW", "rLowS", "rSurfW", "rSurfS"):
        state[n] = g.f[n]
    params.update(params_over or {})   # option variants for parity tests
    return g, params, state, forcing


def cs_global_to_tiles(g, glob, mapIO=1):
    """Global cube-sphere MDS field -> tile layout (..., nTiles, ny, nx), interiors only.
    W2_SET_MAP_TILES (w2_set_map_tiles.F:136-205): W2_mapIO = 1 (compact, data.exch2 of
    solid-body.cs-32x32x1) stacks the facets in y, (..., 6*n, n); W2_mapIO = -1 (the
    default, w2_readparms.F:64, e.g. global_ocean.cs32x15 which has no data.exch2) puts
    them one after the other in x, (..., n, 6*n)."""
    topo = g.topo
    lead = glob.shape[:-2]
    out = np.zeros(lead + (g.nTiles, g.ny, g.nx))
    inner = g.sl(1, g.sNx, 1, g.sNy)
    gNx = glob.shape[-1]
    for t in range(g.nTiles):
        tid = t + 1
        f = topo.face[tid]
        if mapIO == -1:
            x0 = sum(fx for fx, _ in topo.facet_dims[:f - 1]) + topo.tBx[tid]
            y0 = topo.tBy[tid]
        else:
            nb = sum(fx * fy for fx, fy in topo.facet_dims[:f - 1])
            ii = nb + topo.tBx[tid] + topo.tBy[tid] * topo.facet_dims[f - 1][0]
            x0, y0 = ii % gNx, ii // gNx
        out[(Ellipsis, t) + inner] = glob[..., y0:y0 + g.sNy, x0:x0 + g.sNx]
    return out


def solid_body_cs32(data_dir=None):
    """verification/solid-body.cs-32x32x1: cubed sphere, 6 faces of 32x32 (one tile each,
    OL=2, pkg/exch2), 1 level of an ideal-gas atmosphere in p-coordinates (delR=1e5 Pa,
    tRef=300 = theta, so the hydrostatic anomaly is exactly zero), vector-invariant
    momentum, no viscosity, implicit free surface (uniformLin_PhiSurf: Bo_surf =
    1/rhoConst = 1), rotationPeriod=108000, rSphere=5500.4e3 with the grid of radius
    6370e3 rescaled, deltaT=450, abEps=0.1, passive salt (C2 advection) from S_init.bin,
    cg2dTargetResidual=1e-12.  Initial state: code/ini_vel.F (solid-body rotation from
    psi = fac*fCoriG) and code/ini_psurf.F (balanced surface pressure)."""
    from math import pi
    d = data_dir or os.path.join(GOLDEN, "solid-body.cs-32x32x1")
    topo = cube_topology(32, 32, 32, 2)
    g = Grid(32, 32, 2, 2, 1, nSx=6, nSy=1, topology=topo)
    g.usingCurvilinearGrid = True
    g.ini_vertical_grid([1.0e5], Ro_SeaLevel=1.0e5)
    recs = [np.fromfile(os.path.join(d, "tile%03d.mitgrid" % f), dtype=">f8").astype(np.float64).reshape(16, 33, 33)
            for f in range(1, 7)]
    rSphere = 5500.4e3
    g.ini_curvilinear_grid(recs, radius_fromHorizGrid=6370.0e3, rSphere=rSphere, anglesFromFile=False)
    omega = 2.0 * pi / 108000.0
    g.ini_cori(selectCoriMap=2, omega=omega)
    bathy = np.full((g.nTiles, g.ny, g.nx), g.f["rF"][1])     # no bathyFile: R_low = rF(Nr+1)
    g.ini_depths_masks(bathy, hFacMin=1.0, hFacMinDr=0.0, gBaro=9.81)
    rhoConst = 1.0
    g.f["Bo_surf"] = np.full((g.nTiles, g.ny, g.nx), 1.0 / rhoConst)   # ini_linear_phisurf.F, uniformLin_PhiSurf
    g.f["recip_Bo"] = np.full((g.nTiles, g.ny, g.nx), rhoConst)
    g.ini_cg2d(450.0, 450.0, 1e-12)
    params = dict(deltaTMom=450.0, deltaTFreeSurf=450.0, deltaTClock=450.0, deltaTtracer=450.0, abEps=0.1,
                  rhoConst=rhoConst, rhoNil=rhoConst, gravity=9.81, gBaro=9.81, viscAhD=0.0, viscAhZ=0.0,
                  viscA4D=0.0, viscA4Z=0.0, viscAr=0.0, sideDragFactor=2.0, no_slip_sides=0, no_slip_bottom=0,
                  selectCoriScheme=0, vectorInvariantMomentum=1, selectVortScheme=1, selectKEscheme=0,
                  momForcingOutAB=0, momDissip_In_AB=1, cg2dMaxIters=600, cg2dUseMinResSol=0, nIter0=0,
                  exactConserv=0, tempStepping=0, saltStepping=1, saltAdvection=1, saltForcing=1,
                  saltAdvScheme=2, saltVertAdvScheme=2, diffKhS=0.0, diffKrS=0.0, implicitDiffusion=0,
                  ivdc_kappa=0.0, usingCurvilinearGrid=1, rSphere=rSphere, integr_GeoPot=2, gravitySign=1.0,
                  eosType=0, tAlpha=0.0, sBeta=0.0)
    # code/ini_vel.F: psi = fac*fCoriG, full halo range, then EXCH_UV_XYZ_RL(.TRUE.) and masks
    omegaprime = 80.0 / rSphere
    fac = -(rSphere * rSphere) * omegaprime / (2.0 * omega)
    psi = fac * g.f["fCoriG"]
    u = np.zeros((g.nTiles, 1, g.ny, g.nx))
    v = np.zeros_like(u)
    for t in range(g.nTiles):
        for J in range(g.ny):
            Jp = min(J + 1, g.ny - 1)
            for I in range(g.nx):
                Ip = min(I + 1, g.nx - 1)
                u[t, 0, J, I] = 0.0 + (psi[t, J, I] - psi[t, Jp, I]) * g.f["recip_dyG"][t, J, I]
                v[t, 0, J, I] = 0.0 + (psi[t, J, Ip] - psi[t, J, I]) * g.f["recip_dxG"][t, J, I]
    u, v = topo.exchange_uv(u, v, True)
    u = u * g.f["maskW"]
    v = v * g.f["maskS"]
    # code/ini_psurf.F
    psFac = -(rSphere * rSphere) * omegaprime * (omega + omegaprime * 0.5)
    snFac = 1.0 / (4.0 * omega * omega)
    fC = g.f["fCori"]
    etaN = 0.0 + psFac * (snFac * fC * fC - 1.0 / 3.0) * g.f["recip_Bo"]
    salt = cs_global_to_tiles(g, np.fromfile(os.path.join(d, "S_init.bin"), dtype=">f8").astype(np.float64)
                              .reshape(192, 32))[:, None]
    salt = g.exch(salt) * g.f["maskC"]
    state = {"uVel": u, "vVel": v, "etaN": etaN, "salt": salt,
             "theta": np.full((g.nTiles, 1, g.ny, g.nx), 300.0), "tRef": np.array([300.0]),
             "sRef": np.array([0.0])}
    return g, params, state


def advect_cs(data_dir=None, grid_dir=None):
    """verification/advect_cs: cubed sphere, 6 faces of 32x32 (pkg/exch2, code/SIZE.h
    sNx=sNy=32, OL=4, one tile per face), 1 level (delR=1e5, Ro_SeaLevel=1e5: no bathymetry),
    momStepping=F: the solid-body rotation of code/ini_vel.F (psi = fac*fCoriG with
    omegaprime = 38.60328935834681/rSphere) advects theta from T.init with the DST3
    flux-limited multi-dimensional scheme (tempAdvScheme=33: the cube's 3-pass split,
    gad_advection.F:339-367) and GAD_MULTIDIM_COMPRESSIBLE (code/GAD_OPTIONS.h); deltaT=2700,
    no diffusion.  The grid is grid_cs32.faceNNN.bin (input/prepare_run; the same files as
    global_ocean.cs32x15).  Salt uses scheme 80 in the reference and does not feed back: it is
    not stepped here."""
    from math import pi
    d = data_dir or os.path.join(GOLDEN, "advect_cs")
    gd = grid_dir or os.path.join(GOLDEN, "global_ocean.cs32x15")
    n = 32
    topo = cube_topology(n, 32, 32, 4)
    g = Grid(32, 32, 4, 4, 1, nSx=6, nSy=1, topology=topo)
    g.usingCurvilinearGrid = True
    g.ini_vertical_grid([1.0e5], Ro_SeaLevel=1.0e5)
    recs = [np.fromfile(os.path.join(gd, "grid_cs32.face%03d.bin" % f), dtype=">f8").astype(np.float64)
            .reshape(18, n + 1, n + 1) for f in range(1, 7)]
    rSphere = 6370.0e3
    g.ini_curvilinear_grid(recs, radius_fromHorizGrid=6370.0e3, rSphere=rSphere, anglesFromFile=True)
    omega = 2.0 * pi / 86164.0
    g.ini_cori(selectCoriMap=2, omega=omega)
    bathy = np.full((g.nTiles, g.ny, g.nx), g.f["rF"][1])     # no bathyFile: R_low = rF(Nr+1)
    g.ini_depths_masks(bathy, hFacMin=1.0, hFacMinDr=1.0, gBaro=9.81)
    g.ini_cg2d(2700.0, 2700.0, 1e-12)
    params = dict(deltaTMom=2700.0, deltaTFreeSurf=2700.0, deltaTClock=2700.0, deltaTtracer=2700.0, abEps=0.1,
                  rhoConst=999.8, rhoNil=999.8, gravity=9.81, gBaro=9.81, momStepping=0, tempStepping=1,
                  tempAdvection=1, tempForcing=0, tempAdvScheme=33, tempVertAdvScheme=33, multiDimAdvection=1,
                  multiDimCompressible=1, saltStepping=0, diffKhT=0.0, diffKrT=0.0, implicitDiffusion=0,
                  ivdc_kappa=0.0, exactConserv=0, cg2dMaxIters=600, usingCurvilinearGrid=1, rSphere=rSphere,
                  nIter0=0)
    # code/ini_vel.F: psi = fac*fCoriG over the full halo range, EXCH_UV_XYZ_RL(.TRUE.), masks
    omegaprime = 38.60328935834681 / rSphere
    fac = -(rSphere * rSphere) * omegaprime / (2.0 * omega)
    psi = fac * g.f["fCoriG"]
    u = np.zeros((g.nTiles, 1, g.ny, g.nx))
    v = np.zeros_like(u)
    for t in range(g.nTiles):
        for J in range(g.ny):
            Jp = min(J + 1, g.ny - 1)
            for I in range(g.nx):
                Ip = min(I + 1, g.nx - 1)
                u[t, 0, J, I] = 0.0 + (psi[t, J, I] - psi[t, Jp, I]) * g.f["recip_dyG"][t, J, I]
                v[t, 0, J, I] = 0.0 + (psi[t, J, Ip] - psi[t, J, I]) * g.f["recip_dxG"][t, J, I]
    u, v = topo.exchange_uv(u, v, True)
    u = u * g.f["maskW"]
    v = v * g.f["maskS"]
    rd = lambda fn: np.fromfile(os.path.join(d, fn), dtype=">f8").astype(np.float64).reshape(n, 6 * n)
    theta = g.exch(cs_global_to_tiles(g, rd("T.init"), mapIO=-1)[:, None].copy()) * g.f["maskC"]
    salt = g.exch(cs_global_to_tiles(g, rd("S.init"), mapIO=-1)[:, None].copy()) * g.f["maskC"]
    state = {"uVel": u, "vVel": v, "theta": theta, "salt": salt, "tRef": np.array([0.0]), "sRef": np.array([0.0])}
    return g, params, state


CS32_FORCING = {"taux": "trenberth_taux.bin", "tauy": "trenberth_tauy.bin", "Qnet": "shiQnet_cs32.bin",
                "EmPmR": "shiEmPR_cs32.bin", "SST": "lev_surfT_cs_12m.bin", "SSS": "lev_surfS_cs_12m.bin"}


def global_ocean_cs32x15(data_dir=None, sNy=32, params_over=None):
    """verification/global_ocean.cs32x15 (BASELINE config 3): 6 faces of 32x32 on pkg/exch2,
    one 32x32 tile per face at OL=4 (SURVEY 8(d) C3 layout; sNy=16 gives the reference's
    code/SIZE.h tiling sNx=32, sNy=16, nSx=12, two tiles per face), 15 levels,
    curvilinear grid from grid_cs32.faceNNN.bin (18 records incl. AngleCS/SN,
    radius_fromHorizGrid=6370e3), bathy_Hmin50.bin.  input/data: viscAh=3e5, viscAr=1e-3,
    diffKrT=diffKrS=3e-5, ivdc_kappa=10, implicitDiffusion, JMD95Z, staggerTimeStep,
    vectorInvariantMomentum, exactConserv, r* (select_rStar=2, nonlinFreeSurf=4,
    hFacInf=0.2, hFacSup=2), useRealFreshWaterFlux, allowFreezing, hFacMin=0.1,
    hFacMinDr=20, cg2dMaxIters=200, cg2dTargetResWunit=1e-14, deltaTMom=1200,
    deltaTtracer=deltaTFreeSurf=deltaTClock=86400, abEps=0.1, tracForcingOutAB=1, monthly
    periodic forcing, SST/SSS relaxation (5184000 s, 62208000 s), GM-Redi K=800.
    GM-Redi in the advective (bolus stream-function) form, input/data.gmredi GM_AdvForm
    (gmredi_readparms.F:243-250: GM_skewflx = 0, GM_ExtraDiag = GM_isopycK != 0).
    Cold start (nIter0=0) from lev_T/S_cs_15k (the reference restarts from
    pickup.0000072000, which the reference tree does not hold)."""
    d = data_dir or os.path.join(GOLDEN, "global_ocean.cs32x15")
    n, Nr = 32, 15
    topo = cube_topology(n, 32, sNy, 4)
    g = Grid(32, sNy, 4, 4, Nr, nSx=topo.nTiles, nSy=1, topology=topo)
    g.usingCurvilinearGrid = True
    g.ini_vertical_grid(LATLON_DELR)
    recs = [np.fromfile(os.path.join(d, "grid_cs32.face%03d.bin" % f), dtype=">f8").astype(np.float64)
            .reshape(18, n + 1, n + 1) for f in range(1, 7)]
    g.ini_curvilinear_grid(recs, radius_fromHorizGrid=6370.0e3, rSphere=6370.0e3, anglesFromFile=True)
    g.ini_cori(selectCoriMap=2)
    rd = lambda fn, shp: np.fromfile(os.path.join(d, fn), dtype=">f8").astype(np.float64).reshape(shp)
    bathy = cs_global_to_tiles(g, rd("bathy_Hmin50.bin", (n, 6 * n)), mapIO=-1)   # no data.exch2
    g.ini_depths_masks(bathy, hFacMin=0.1, hFacMinDr=20.0, gBaro=9.81)
    g.ini_cg2d(1200.0, 86400.0, 1e-7, cg2dTargetResWunit=1e-14)
    rhoConstFresh = 1000.0
    forcing = {}
    for name, fn in CS32_FORCING.items():
        rec = np.moveaxis(cs_global_to_tiles(g, rd(fn, (12, n, 6 * n)), mapIO=-1), 0, 1).copy()   # (nTiles, 12, ny, nx)
        if name == "EmPmR":
            rec = rec * rhoConstFresh
        if name in ("taux", "tauy"):
            forcing[name] = rec
        else:
            forcing[name] = np.moveaxis(g.exch(rec), 1, 0).copy()
    fu, fv = topo.exchange_uv(forcing.pop("taux"), forcing.pop("tauy"), True)   # EXCH_UV_XY_RS(fu,fv,.TRUE.)
    forcing["taux"], forcing["tauy"] = np.moveaxis(fu, 1, 0).copy(), np.moveaxis(fv, 1, 0).copy()
    mC = g.f["maskC"]
    theta = g.exch(cs_global_to_tiles(g, rd("lev_T_cs_15k.bin", (Nr, n, 6 * n)), mapIO=-1).swapaxes(0, 1).copy())
    theta[mC == 0.0] = 0.0
    theta = np.where(theta < -1.9, -1.9, theta)         # ini_theta.F: checkIniTemp .AND. allowFreezing
    salt = g.exch(cs_global_to_tiles(g, rd("lev_S_cs_15k.bin", (Nr, n, 6 * n)), mapIO=-1).swapaxes(0, 1).copy())
    salt[mC == 0.0] = 0.0
    params = dict(deltaTMom=1200.0, deltaTFreeSurf=86400.0, deltaTClock=86400.0, deltaTtracer=86400.0,
                  abEps=0.1, rhoConst=1035.0, rhoConstFresh=rhoConstFresh, gravity=9.81,
                  gBaro=9.81, viscAhD=3e5, viscAhZ=3e5, viscA4D=0.0, viscA4Z=0.0, viscAr=1e-3,
                  sideDragFactor=2.0, selectCoriScheme=0, vectorInvariantMomentum=1, selectVortScheme=1,
                  selectKEscheme=0, momForcingOutAB=0, momDissip_In_AB=1, cg2dMaxIters=200, cg2dUseMinResSol=0,
                  nIter0=0, no_slip_sides=1, no_slip_bottom=1, exactConserv=1, staggerTimeStep=1,
                  tracForcingOutAB=1, tempStepping=1, tempAdvection=1, tempForcing=1, tempAdvScheme=2,
                  tempVertAdvScheme=2, saltStepping=1, saltAdvection=1, saltForcing=1, saltAdvScheme=2,
                  saltVertAdvScheme=2, diffKhT=0.0, diffKrT=3e-5, diffKhS=0.0, diffKrS=3e-5,
                  ivdc_kappa=10.0, implicitDiffusion=1, usingCurvilinearGrid=1, rSphere=6370.0e3,
                  integr_GeoPot=2, eosType=1, allowFreezing=1, useRealFreshWaterFlux=1, HeatCapacity_Cp=3994.0,
                  convertFW2Salt=-1.0, temp_EvPrRn=123456.7, salt_EvPrRn=0.0, periodicExternalForcing=1,
                  externForcingPeriod=2592000.0, externForcingCycle=31104000.0, useGMRedi=1,
                  GM_background_K=800.0, GM_isopycK=800.0, GM_skewflx=0.0, GM_AdvForm=1, GM_ExtraDiag=1,
                  GM_maxSlope=1e-2,
                  GM_Kmin_horiz=50.0, nonlinFreeSurf=4, select_rStar=2, hFacInf=0.2, hFacSup=2.0,
                  cg2dPreCondFreq=1)
    pRef = np.array([0.0 + 1035.0 * (g.f["rC"][k] - g.f["rF"][0]) * 9.81 * -1.0 for k in range(Nr)])
    rC, rF = g.f["rC"], g.f["rF"]
    phiRef = np.zeros(2 * Nr + 1)
    for k in range(Nr):
        phiRef[2 * k + 1] = phiRef[0] + (rC[k] - rF[0]) * 9.81 * -1.0
        phiRef[2 * k + 2] = phiRef[0] + (rF[k + 1] - rF[0]) * 9.81 * -1.0
    lamT = np.full((g.nTiles, g.ny, g.nx), 1.0 / 5184000.0)
    lamS = np.full((g.nTiles, g.ny, g.nx), 1.0 / 62208000.0)
    state = {"theta": theta, "salt": salt, "tRef": np.full(Nr, 20.0), "sRef": np.full(Nr, 35.0),
             "pRef4EOS": pRef, "phiRef": phiRef, "lambdaThetaClimRelax": lamT, "lambdaSaltClimRelax": lamS,
             "fu": forcing["taux"][0], "fv": forcing["tauy"][0], "Qnet": forcing["Qnet"][0],
             "EmPmR": forcing["EmPmR"][0], "SST": forcing["SST"][0], "SSS": forcing["SSS"][0]}
    for nm in ("h0FacC", "h0FacW", "h0FacS", "recip_Rcol", "rLowW", "rLowS", "rSurfW", "rSurfS"):
        state[nm] = g.f[nm]
    params.update(params_over or {})   # option variants for parity tests
    return g, params, state, forcing


def llc_delr(Nr):
    """Synthetic vertical grid of the LLC workload: delR growing linearly from 10 m to
    160 m (Nr = 50: 4 250 m in all)."""
    return [10.0 + 150.0 * k / max(1, Nr - 1) for k in range(Nr)]


def llc_synthetic(n=90, Nr=50, OL=4, tile=None, seed=20261015):
    """BASELINE config 5, the LLC-90-shaped synthetic of SURVEY.md 8(d): the 5 facets of
    utils/exch2/input/data.exch2.llc_120_5f with 120 -> n (n x 3n, n x 3n, n x n, 3n x n,
    3n x n), tiles of `tile` x `tile` (default n: 13 tiles), Nr levels, OL halo rows.
      grid       uniform curvilinear metrics dx = dy = 1e5 m on every facet (the facet
                 links carry the rotations), f-plane f0 = 1e-4;
      bathymetry H = -4000 (0.6 + 0.4 cos(pi r)), r the facet-normalised distance from the
                 facet centre, land on the open edges (south of facets 1, 2, east of 4, 5);
      state      T = tRef(k) + 0.01 N(0,1), S = 35 + 0.001 N(0,1) (numpy default_rng(seed)),
                 u = v = 0, eta = 0;
      forcing    zonal (facet-x) wind stress -0.1 cos(2 pi y / L_y), facet coordinates;
      physics    vector-invariant momentum (harmonic viscosity 1e4), linear free surface with
                 exactConserv, LINEAR EOS, C2 tracers with implicit vertical diffusion and
                 IVDC, deltaT = 3600 s (1/24 model day per step).
    Returns (grid, params, state)."""
    from math import cos, pi, sqrt
    from .exch2 import llc_topology
    ts = tile or n
    topo = llc_topology(n, ts, ts, OL)
    g = Grid(ts, ts, OL, OL, Nr, nSx=topo.nTiles, nSy=1, topology=topo)
    g.usingCurvilinearGrid = True
    g.ini_vertical_grid(llc_delr(Nr))
    dx = 1.0e5
    recs, bath_f, wind_f = [], [], []
    for (fNx, fNy) in topo.facet_dims:
        r = np.zeros((18, fNy + 1, fNx + 1))
        jj, ii = np.meshgrid(np.arange(fNy + 1, dtype=np.float64), np.arange(fNx + 1, dtype=np.float64),
                             indexing="ij")
        r[0], r[1] = (ii + 0.5) * dx, (jj + 0.5) * dx        # XC, YC (m)
        r[5], r[6] = ii * dx, jj * dx                        # XG, YG
        for q in (2, 3, 7, 8, 10, 11, 14, 15):               # DXF DYF DXV DYU DXC DYC DXG DYG
            r[q] = dx
        for q in (4, 9, 12, 13):                             # RA RAZ RAW RAS
            r[q] = dx * dx
        r[16], r[17] = 1.0, 0.0                              # AngleCS, AngleSN
        recs.append(r)
        # bathymetry and wind on the facet's cell centres
        yc, xc = np.meshgrid(np.arange(fNy) + 0.5, np.arange(fNx) + 0.5, indexing="ij")
        rr = np.sqrt(((xc - fNx / 2.0) / (fNx / 2.0)) ** 2 + ((yc - fNy / 2.0) / (fNy / 2.0)) ** 2) / sqrt(2.0)
        bath_f.append(-4000.0 * (0.6 + 0.4 * np.cos(pi * rr)))
        wind_f.append(-0.1 * np.cos(2.0 * pi * yc / fNy))
    # land on the disconnected (Antarctic) edges
    bath_f[0][0, :] = 0.0
    bath_f[1][0, :] = 0.0
    bath_f[3][:, -1] = 0.0
    bath_f[4][:, -1] = 0.0
    g.ini_curvilinear_grid(recs, radius_fromHorizGrid=6370.0e3, rSphere=6370.0e3, anglesFromFile=True)
    g.ini_cori(1.0e-4, 0.0, selectCoriMap=0)
    g.f["fCoriCos"] = g.z2()

    def facet_to_tiles(fld):
        out = g.z2()
        inner = g.sl(1, g.sNx, 1, g.sNy)
        for t in range(g.nTiles):
            tid = t + 1
            f = topo.face[tid]
            out[t][inner] = fld[f - 1][topo.tBy[tid]:topo.tBy[tid] + g.sNy, topo.tBx[tid]:topo.tBx[tid] + g.sNx]
        return out
    g.ini_depths_masks(facet_to_tiles(bath_f), hFacMin=0.1, hFacMinDr=20.0, gBaro=9.81)
    dt = 3600.0
    g.ini_cg2d(dt, dt, 1e-9)
    rC = g.f["rC"][:Nr]
    tRef = 2.0 + 18.0 * np.exp(rC / 1000.0)
    rng = np.random.default_rng(seed)
    shape = (g.nTiles, Nr, g.ny, g.nx)
    theta = tRef[None, :, None, None] + 0.01 * rng.standard_normal(shape)
    salt = 35.0 + 0.001 * rng.standard_normal(shape)
    mC = g.f["maskC"]
    theta = g.exch(np.where(mC > 0.0, theta, 0.0))
    salt = g.exch(np.where(mC > 0.0, salt, 0.0))
    fu = facet_to_tiles(wind_f)
    fu, fv = topo.exchange_uv(fu[:, None], g.z2()[:, None], True)
    params = dict(deltaTMom=dt, deltaTFreeSurf=dt, deltaTClock=dt, deltaTtracer=dt, abEps=0.1, rhoConst=1035.0,
                  rhoNil=1035.0, gravity=9.81, gBaro=9.81, viscAhD=1.0e4, viscAhZ=1.0e4, viscA4D=0.0, viscA4Z=0.0,
                  viscAr=1.0e-4, sideDragFactor=2.0, selectCoriScheme=0, vectorInvariantMomentum=1,
                  selectVortScheme=1, selectKEscheme=0, momForcingOutAB=0, momDissip_In_AB=1, cg2dMaxIters=1000,
                  cg2dUseMinResSol=0, nIter0=0, no_slip_sides=1, no_slip_bottom=1, exactConserv=1,
                  tempStepping=1, tempAdvection=1, tempForcing=1, tempAdvScheme=2, tempVertAdvScheme=2,
                  saltStepping=1, saltAdvection=1, saltForcing=1, saltAdvScheme=2, saltVertAdvScheme=2,
                  diffKhT=0.0, diffKrT=1.0e-5, diffKhS=0.0, diffKrS=1.0e-5, ivdc_kappa=10.0, implicitDiffusion=1,
                  usingCurvilinearGrid=1, rSphere=6370.0e3, integr_GeoPot=2, eosType=0, tAlpha=2.0e-4, sBeta=7.4e-4)
    state = {"theta": theta, "salt": salt, "tRef": tRef, "sRef": np.full(Nr, 35.0), "fu": fu[:, 0], "fv": fv[:, 0]}
    return g, params, state
