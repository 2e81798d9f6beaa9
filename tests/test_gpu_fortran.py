"""The Fortran side of the drop-in boundary on the GPU: mitgcm_amd/fortran/fhost, a
Fortran host that owns every array (as the reference's COMMON blocks do), registers them
with MGCM_AMD_BIND and steps FORWARD_STEP's routine sequence through the drop-ins
(DO_OCEANIC_PHYS_AMD, THERMODYNAMICS_AMD, DYNAMICS_AMD, SOLVE_FOR_PRESSURE_AMD,
MOMENTUM_CORRECTION_STEP_AMD, INTEGR_CONTINUITY_AMD, DO_FIELDS_BLOCKING_EXCHANGES_AMD),
with the host computing EXTERNAL_FIELDS_LOAD itself.

Bars:
  * the state after N steps is bit-identical to the device-resident, graph-captured path
    (Model.forward_step) on the same configuration -- BASELINE config 2 (global_ocean
    90x40x15, monthly forcing, GM/Redi) and config 4 (baroclinic gyre, 4 tiles, DST3-FL);
  * EXCH_XYZ_RL / EXCH_UV_XYZ_RL / EXCH_XY_RL on host arrays whose halos were overwritten
    rebuild exactly the exchanged halos;
  * GLOBAL_SUM_TILE_RL is the tile-ordered sum (global_sum_tile.F:150-156).
"""
import os
import subprocess

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FHOST = os.path.join(ROOT, "mitgcm_amd", "fortran", "fhost")
FORCING = ("fu", "fv", "Qnet", "EmPmR", "SST", "SSS")
CHECK = ("uVel", "vVel", "wVel", "theta", "salt", "etaN", "etaH", "gU", "gV", "guNm1", "gvNm1", "gtNm1", "gsNm1",
         "rhoInSitu", "surfaceForcingT", "Kwx", "totPhiHyd")


def _name(s):
    return s.encode().ljust(32)


def _write_blob(path, m, nsteps):
    from mitgcm_amd._lib import lib
    from mitgcm_amd.model import GRID_1D, GRID_2D, GRID_3D, STATE_1D, STATE_2D, STATE_3D
    L, g = lib(), m.g
    names, i = [], 0
    while L.mgcm_param_name(i):
        names.append(L.mgcm_param_name(i).decode())
        i += 1
    params = {n: L.mgcm_get_param(m.h, n.encode()) for n in names}
    # options the device reads at set-up beyond its parameter table (usingSphericalPolarGrid,
    # rSphere, selectMetricTerms, integr_GeoPot, the vertical advection schemes, ...)
    for n, v in m.params.items():
        params.setdefault(n, float(v))
    periodic = int(params["periodicExternalForcing"])
    nRec = int(params["nForcRec"]) if periodic else 0
    params["periodicExternalForcing"] = 0.0     # the host loads the forcing (LOAD_FIELDS_DRIVER)
    operator = ("aW2d", "aS2d", "aC2d", "pW", "pS", "pC")
    fields = [(n, 1) for n in GRID_1D] + [(n, 0) for n in STATE_1D]
    fields += [(n, 0 if n in operator else 1) for n in GRID_2D] + [(n, 0) for n in STATE_2D]
    fields += [(n, 0) for n in GRID_3D + STATE_3D]
    # what the host's LOAD_FIELDS_DRIVER writes every step: host input (kind 2)
    fields = [(n, 2 if n in FORCING else st) for n, st in fields]
    with open(path, "wb") as fh:
        fh.write(np.array([g.sNx, g.sNy, g.OLx, g.OLy, g.Nr, g.nSx, g.nSy, len(params), len(fields), nsteps,
                           int(params["nIter0"]), nRec, periodic], dtype=np.int32).tobytes())
        fh.write(np.array([params["deltaTClock"], params["externForcingPeriod"],
                           params["externForcingCycle"]]).tobytes())
        for n, v in params.items():
            fh.write(_name(n) + np.float64(v).tobytes())
        for n, st in fields:
            a = np.ascontiguousarray(m.get(n), dtype=np.float64).reshape(-1)
            fh.write(_name(n) + np.array([a.size, st], dtype=np.int32).tobytes() + a.tobytes())
        if periodic:
            fh.write(np.ascontiguousarray(m.get("forcRec").reshape(-1)[:6 * nRec * g.nTiles * g.nx * g.ny]).tobytes())
    return [n for n, st in fields if not st]


def _read_out(path, g, state_names):
    raw = open(path, "rb").read()
    n2 = g.nTiles * g.nx * g.ny
    n3 = n2 * g.Nr
    off = 0

    def take(n):
        nonlocal off
        a = np.frombuffer(raw, dtype=np.float64, count=n, offset=off)
        off += 8 * n
        return a
    out = {"exch_theta": take(n3), "exch_u": take(n3), "exch_v": take(n3), "exch_xy": take(n2),
           "tile": take(g.nTiles), "sum": take(1)[0]}
    for _ in state_names:
        name = raw[off:off + 32].decode().strip()
        cnt = int(np.frombuffer(raw, dtype=np.int32, count=1, offset=off + 32)[0])
        off += 36
        out[name] = take(cnt)
    assert off == len(raw)
    return out


@pytest.mark.parametrize("cfg,nsteps", [("ocean90", 4), ("gyre", 4)])
def test_fortran_host_forward_step_bitexact(cfg, nsteps, tmp_path):
    from mitgcm_amd import configs
    assert os.path.exists(FHOST), "mitgcm_amd/fortran/fhost not built (__graft_entry__.build())"

    def make():
        if cfg == "gyre":
            return configs.make_model(configs.baroclinic_gyre, tempAdvScheme=33)
        return configs.make_model(configs.global_ocean_90x40x15)
    m = make()
    g = m.g
    state = _write_blob(tmp_path / "fhost_in.bin", m, nsteps)
    r = subprocess.run([FHOST, str(tmp_path)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    out = _read_out(tmp_path / "fhost_out.bin", g, state)
    m.forward_step(nsteps)
    m.sync()
    bad = []
    for n in CHECK:
        dev = m.get(n).reshape(-1)
        if not np.array_equal(out[n], dev):
            bad.append((n, float(np.abs(out[n] - dev).max())))
    assert not bad, bad
    # halo points the topology's EXCH does not write keep fhost's marker (-999)
    theta, u, v = m.get("theta"), m.get("uVel"), m.get("vVel")
    src = g.topo.src_of_point()

    def same(host, dev, nz):
        dev = np.moveaxis(dev.reshape(g.nTiles, nz, g.ny * g.nx), 1, 0).reshape(nz, -1)
        host = np.moveaxis(host.reshape(g.nTiles, nz, g.ny * g.nx), 1, 0).reshape(nz, -1)
        untouched = src == np.arange(src.size)
        halo = np.zeros(src.size, bool)
        ii = np.arange(g.nx)
        jj = np.arange(g.ny)
        inter = ((ii[None, :] >= g.OLx) & (ii[None, :] < g.OLx + g.sNx) &
                 (jj[:, None] >= g.OLy) & (jj[:, None] < g.OLy + g.sNy)).reshape(-1)
        halo[:] = ~np.tile(inter, g.nTiles)
        marker = halo & untouched
        ok = np.array_equal(host[:, ~marker], dev[:, ~marker]) and np.all(host[:, marker] == -999.0)
        return ok, int((host[:, ~marker] != dev[:, ~marker]).sum()), int(marker.sum())
    r1 = same(out["exch_theta"], theta, g.Nr)
    assert r1[0], ("EXCH_XYZ_RL", r1)
    r2 = same(out["exch_u"], u, g.Nr), same(out["exch_v"], v, g.Nr)
    assert r2[0][0] and r2[1][0], ("EXCH_UV_XYZ_RL", r2)
    r3 = same(out["exch_xy"], np.ascontiguousarray(theta[:, 0]), 1)
    assert r3[0], ("EXCH_XY_RL", r3)
    inner = (slice(None), 0) + g.sl(1, g.sNx, 1, g.sNy)
    tiles = np.array([theta[t][inner[1:]].sum() for t in range(g.nTiles)])   # per-tile, as fhost sums
    s = 0.0
    for t in range(g.nTiles):
        s = s + out["tile"][t]
    assert out["sum"] == s and np.allclose(out["tile"], tiles, rtol=1e-13, atol=0)
    m.close()
