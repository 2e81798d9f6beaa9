"""The drop-in boundary run the way a reference build runs it: mitgcm_amd/fortran/refhost
(mitgcm_amd/fortran/build_refhost.py) is compiled against the reference's own headers, so
the model state lives in the reference's COMMON blocks (DYNVARS.h, GRID.h, SURFACE.h,
FFIELDS.h, CG2D.h, GMREDI.h, ...), and steps FORWARD_STEP's routine sequence by calling
the MODS shims under their reference names -- DO_OCEANIC_PHYS(myTime, myIter, myThid),
THERMODYNAMICS, DYNAMICS, UPDATE_R_STAR(.TRUE., ...), UPDATE_CG2D, SOLVE_FOR_PRESSURE,
MOMENTUM_CORRECTION_STEP, INTEGR_CONTINUITY(uVel, vVel, ...), CALC_R_STAR(etaH, ...),
DO_FIELDS_BLOCKING_EXCHANGES(myThid) -- with its own EXTERNAL_FIELDS_LOAD in between.  So
MGCM_AMD_MIRROR binds the COMMON blocks and runs, with eosType = 'JMD95P' (BASELINE
config 2's EOS), and the mirror is device-authoritative inside the time loop.  The run-time
parameters are the experiment's own namelist files (input/data, data.pkg, data.gmredi)
resolved by refhost (refhost_parms.F, pinned against the reference's own parameter dump by
tests/test_refhost_params.py) -- not the device model's table; the harness input carries
the arrays and the run's control only.

Bars, BASELINE config 2 (global_ocean.90x40x15 from its pickups):
  * on the reference's SIZE.h (9 x 4 tiles of 10 x 10), with the performance CG2D and with
    cg2dRefOrder (the order results/output.txt was summed in, tests/test_gpu_refpin.py),
    and on one 90 x 40 tile: the state after 6 steps through the MODS drop-ins is
    bit-identical to the device-resident, graph-replayed mgcm_forward_step;
  * the same with the 36 tiles over 2, 3 and 4 device models of the one host process
    (MGCM_AMD_MODELS: tiles over GPUs, the models' halo sources and right-hand-side / free-
    surface blocks copied between them at the reference's exchange points), with the gathered
    single-CU CG2D and with the device-sharded multi-workgroup CG2D: bit-identical to one model;
  * with one model, the steps after the first run as ONE graph replay each at their
    DO_OCEANIC_PHYS (the recorded FORWARD_STEP order, the forcing uploaded first), still
    bit-identical; MGCM_AMD_EAGER=1 keeps the routine-by-routine path, tested too;
  * the mirror moves the state down only after the steps a host routine reads
    (monitorFreq = 2 days, nEndIter) -- 3 of 6 -- and otherwise only the 6 forcing fields up;
  * ms/step through the drop-ins is recorded beside the graph path's.
"""
import json
import os
import subprocess
import sys
import time

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
RH = os.path.join(ROOT, "mitgcm_amd", "fortran", "refhost")
CHECK = ("uVel", "vVel", "wVel", "theta", "salt", "etaN", "etaH", "gU", "gV", "guNm1", "gvNm1", "gtNm1", "gsNm1",
         "rhoInSitu", "totPhiHyd", "hFacC", "hFacW", "rStarFacC", "aW2d", "pC", "uVelD", "etaNm1", "Kwx", "dEtaHdt")
NSTEPS = 6


def _mirror_calls(undef=()):
    sys.path.insert(0, os.path.join(ROOT, "mitgcm_amd", "fortran"))
    import build_refhost
    return build_refhost.mirror_calls(undef)


def _name(s):
    return s.encode().ljust(32)


# The experiment's own namelist files (verification/global_ocean.90x40x15/input: data,
# data.pkg, data.gmredi, fixtures): refhost reads its run-time parameters from them
# (refhost_parms.F), never from the device model's table or configs.py.
PARAM_DIR = os.path.join(ROOT, "tests", "golden", "global_ocean.90x40x15", "input")


def _write_blob(path, m, nsteps, monitor_days, packages_off=True, extra=(), w2=None, undef=()):
    """refhost_in.bin: sizes, the run's control (the only parameters it carries: the run length,
    the monitor schedule, and -- packages_off -- pkg/sbo and pkg/diagnostics switched off for
    the run), the COMMON-block arrays (grid, masks and the restart state), the forcing records
    and -- w2, a pkg/exch2 topology (Exch2Topology.w2_arrays at W2_EXCH2_SIZE.h's leading
    dimensions) -- the W2_EXCH2_TOPOLOGY.h arrays (refhost.F REFHOST_W2_READ)."""
    g = m.g
    _, fields = _mirror_calls(undef)
    dtc = m.params["deltaTClock"]
    nIter0 = int(m.params["nIter0"])
    params = [("monitorFreq", monitor_days * dtc), ("nEndIter", float(nIter0 + nsteps))]
    if packages_off:
        params += [("useSBO", 0.0), ("useDiagnostics", 0.0)]
    params += list(extra)
    periodic = int(m.params.get("periodicExternalForcing", 0))
    nRec = int(m.params.get("nForcRec", 12)) if periodic else 0
    blob_fields = []
    for n, kind in fields:
        if n == "phiRef":      # phiRef(2*Nr+1) of set_ref_state.F; the device holds phiRef(2k)
            a = np.zeros(2 * g.Nr + 1)
            a[1::2] = m.get("phiRefC").reshape(-1)[:g.Nr]
        else:
            a = np.ascontiguousarray(m.get(n), dtype=np.float64).reshape(-1)
        blob_fields.append((n, kind, a))
    with open(path, "wb") as fh:
        fh.write(np.array([g.sNx, g.sNy, g.OLx, g.OLy, g.Nr, g.nSx, g.nSy, len(params), len(blob_fields), nsteps,
                           nIter0, nRec, periodic, g.nTiles if w2 else 0], dtype=np.int32).tobytes())
        fh.write(np.array([dtc, m.params.get("externForcingPeriod", 0.0),
                           m.params.get("externForcingCycle", 0.0)]).tobytes())
        for n, v in params:
            fh.write(_name(n) + np.float64(v).tobytes())
        for n, kind, a in blob_fields:
            fh.write(_name(n) + np.array([a.size, kind], dtype=np.int32).tobytes() + a.tobytes())
        if periodic:
            fh.write(np.ascontiguousarray(m.get("forcRec").reshape(-1)[:6 * nRec * g.nTiles * g.nx * g.ny]).tobytes())
        if w2:
            fh.write(np.array([w2["ldNb"], w2["ldT"]], dtype=np.int32).tobytes())
            for k in ("myFace", "tBasex", "tBasey", "isNedge", "isSedge", "isEedge", "isWedge", "nNeighbours",
                      "neighbourId", "opposingSend", "neighbourDir", "pij", "oi", "oj", "iLo", "iHi", "jLo", "jHi"):
                fh.write(np.ascontiguousarray(w2["exch2_" + k], dtype=np.int32).tobytes())
    return [n for n, k, a in blob_fields if k == 0]


def _read_out(path, state_names, nsteps):
    raw = open(path, "rb").read()
    nfs, nup, ndown = np.frombuffer(raw, dtype=np.int32, count=3)
    secs, bup, bdown = np.frombuffer(raw, dtype=np.float64, count=3, offset=12)
    step_s = np.frombuffer(raw, dtype=np.float64, count=nsteps, offset=36)
    off = 36 + 8 * nsteps
    out = {}
    for _ in state_names:
        name = raw[off:off + 32].decode().strip()
        cnt = int(np.frombuffer(raw, dtype=np.int32, count=1, offset=off + 32)[0])
        off += 36
        out[name] = np.frombuffer(raw, dtype=np.float64, count=cnt, offset=off)
        off += 8 * cnt
    assert off == len(raw)
    return out, {"steps_timed": int(nfs), "uploads": int(nup), "downloads": int(ndown), "seconds": float(secs),
                 "bytes_up": float(bup), "bytes_down": float(bdown), "step_ms": [1e3 * x for x in step_s]}


# models > 1: the host's 36 tiles over that many device models (MGCM_AMD_MODELS; all on the
# one GPU of the test box), stepped through the same drop-ins with the models' halo sources,
# right-hand-side blocks and free-surface blocks copied between them at the reference's
# exchange points (fortran_abi.hip); mwg = 1: the device-sharded multi-workgroup CG2D
# (MGCM_CG2D_MWG) instead of the gathered single-CU solve
# eager = 1: every step routine by routine (MGCM_AMD_EAGER); otherwise, with one model, the
# steps after the first run as one graph replay each (fortran_abi.hip: the first
# device-authoritative step is recorded in FORWARD_STEP's order, later ones replay it)
# packages = 1: data.pkg as the experiment has it -- pkg/sbo and pkg/diagnostics read the
# state every step, so it comes down after every step (MGCM_AMD_DIAGNOSTICS=state: state
# diagnostics only; the mirror refuses useDiagnostics otherwise)
@pytest.mark.parametrize("layout,refOrder,models,mwg,eager,packages", [
    ("ref", 0, 1, 0, 0, 0), ("ref", 1, 1, 0, 0, 0), ("1t", 0, 1, 0, 0, 0), ("1t", 0, 1, 0, 1, 0),
    ("ref", 0, 1, 0, 1, 0), ("ref", 0, 2, 0, 0, 0), ("ref", 0, 4, 0, 1, 0), ("ref", 0, 4, 0, 0, 0), ("ref", 1, 4, 0, 0, 0),
    ("ref", 0, 1, 1, 0, 0), ("ref", 0, 3, 1, 0, 0), ("1t", 0, 1, 0, 0, 1)])
def test_refhost_mods_dropins_bitexact(layout, refOrder, models, mwg, eager, packages, tmp_path):
    from mitgcm_amd import configs
    exe = os.path.join(RH, "refhost_" + layout)
    assert os.path.exists(exe), "refhost not built (mitgcm_amd/fortran/build_refhost.py, __graft_entry__.build())"
    tiles = {"ref": (9, 4), "1t": (1, 1)}[layout]

    def cfg():
        g, params, state, forcing = configs.global_ocean_90x40x15(nSx=tiles[0], nSy=tiles[1])
        params["cg2dRefOrder"] = refOrder
        if mwg:
            params["cg2dForceMwg"] = 1
        return g, params, state, forcing
    m = configs.make_model(cfg)
    state = _write_blob(tmp_path / "refhost_in.bin", m, NSTEPS, monitor_days=2, packages_off=not packages)
    env = dict(os.environ, MGCM_CG2D_REFORDER=str(refOrder), MGCM_AMD_MODELS=str(models), MGCM_CG2D_MWG=str(mwg),
               MGCM_AMD_EAGER=str(eager))
    if packages:
        env["MGCM_AMD_DIAGNOSTICS"] = "state"
    r = subprocess.run([exe, str(tmp_path), PARAM_DIR], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stdout + r.stderr
    out, st = _read_out(tmp_path / "refhost_out.bin", state, NSTEPS)
    # the same configuration stepped by the graph-replayed resident path
    m.forward_step(1)     # warm (first step)
    m.prepare()           # graphs built, overlap trial done: outside the timed steps
    m.sync()
    t0 = time.perf_counter()
    m.forward_step(NSTEPS - 1)
    m.sync()
    graph_ms = 1e3 * (time.perf_counter() - t0) / (NSTEPS - 1)
    bad = []
    for n in CHECK:
        if n not in out:
            continue
        dev = m.get(n).reshape(-1)[:out[n].size]
        if not np.array_equal(out[n], dev):
            bad.append((n, float(np.abs(out[n] - dev).max())))
    m.close()
    ms = 1e3 * st["seconds"] / max(1, st["steps_timed"])
    # steps 3 and 5 end without a host reader: no state download, only the forcing upload
    quiet = [st["step_ms"][i] for i in (2, 4)]
    rec = {"layout": layout, "cg2dRefOrder": refOrder, "models": models, "cg2dForceMwg": mwg, "eager": eager,
           "packages": packages,
           "dropin_ms_per_step_mean": ms,
           "dropin_ms_per_step_no_download": float(np.mean(quiet)), "graph_ms_per_step": graph_ms,
           "mirror": st, "state_fields": len(state)}
    print("refhost %s refOrder=%d models=%d mwg=%d eager=%d: %s" % (layout, refOrder, models, mwg, eager,
                                                                   json.dumps(rec)))
    if os.path.isdir(os.path.join(ROOT, "gpurun_out")):
        with open(os.path.join(ROOT, "gpurun_out", "refhost_%s_%d_m%d_w%d_e%d_p%d.json" % (
                layout, refOrder, models, mwg, eager, packages)), "w") as f:
            json.dump(rec, f)
    assert not bad, bad
    assert len([n for n in CHECK if n in out]) >= 20
    # the state came down after steps 2, 4 and 6 only (monitorFreq = 2 days, nEndIter = 6),
    # or after every step when pkg/sbo and pkg/diagnostics read it (packages)
    assert st["downloads"] == (NSTEPS if packages else 3) * len(state), (st, len(state))


# Throughput of the drop-in path over a longer run: 60 steps, every step after the recorded
# one a replay whose forcing goes up in stream order (mgcm_put_async) while the previous step
# still runs -- no per-step fence (MGCM_AMD_STEP_FENCE=0), so the host's Fortran side of step
# n+1 overlaps the device's step n.  io = "namelist": the experiment's own output schedule
# (dumpFreq = 10 days: the state comes down after every 10th step, into the registered COMMON
# pages); io = "off": dumpFreq = 0, the state comes down after the last step only.  The state
# after the run is bit-identical to the resident graph path's; both rates are recorded
# (INTEGRATION.md section 3).  models > 1: the 36 tiles over that many device models of the
# one GPU, every step after the recorded one ONE replay of the graph captured across the
# models' own streams (the default from 4 models on, cap = "multi") or with every model on model
# 0's stream (the default below 4, cap = "one"); cap = "virtual": the models stand for that
# many GPUs, all on device 0 (MGCM_AMD_DEVICES=virtual) -- the per-GPU segment graphs, or
# routine by routine ("virtual-eager").
@pytest.mark.parametrize("io,register,models,cap", [("namelist", 1, 1, ""), ("off", 1, 1, ""), ("namelist", 0, 1, ""),
                                                    ("off", 1, 2, ""), ("off", 1, 3, ""), ("off", 1, 4, ""),
                                                    ("off", 1, 6, ""), ("off", 1, 2, "multi"), ("off", 1, 4, "one"),
                                                    ("off", 1, 6, "one"), ("off", 1, 3, "multi"), ("off", 1, 2, "virtual"),
                                                    ("off", 1, 4, "virtual"), ("off", 1, 4, "virtual-eager")])
def test_refhost_dropin_throughput(io, register, models, cap, tmp_path):
    from mitgcm_amd import configs
    nsteps = 60
    exe = os.path.join(RH, "refhost_ref")
    assert os.path.exists(exe), "refhost not built (mitgcm_amd/fortran/build_refhost.py, __graft_entry__.build())"
    m = configs.make_model(lambda: configs.global_ocean_90x40x15(nSx=9, nSy=4))
    extra = [("dumpFreq", 0.0)] if io == "off" else []
    state = _write_blob(tmp_path / "refhost_in.bin", m, nsteps, monitor_days=10 * nsteps, extra=extra)
    env = dict(os.environ, MGCM_AMD_MODELS=str(models), MGCM_AMD_EAGER="0", MGCM_AMD_STEP_FENCE="0",
               MGCM_AMD_REGISTER=str(register), MGCM_AMD_CAPTURE=cap if cap in ("one", "multi") else "")
    if cap.startswith("virtual"):
        env.update(MGCM_AMD_DEVICES="virtual", MGCM_AMD_EAGER="1" if cap == "virtual-eager" else "0")
    r = subprocess.run([exe, str(tmp_path), PARAM_DIR], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stdout + r.stderr
    out, st = _read_out(tmp_path / "refhost_out.bin", state, nsteps)
    m.forward_step(1)
    m.prepare()
    m.sync()
    t0 = time.perf_counter()
    m.forward_step(nsteps - 1)
    m.sync()
    graph_ms = 1e3 * (time.perf_counter() - t0) / (nsteps - 1)
    bad = [(n, float(np.abs(out[n] - m.get(n).reshape(-1)[:out[n].size]).max())) for n in CHECK
           if n in out and not np.array_equal(out[n], m.get(n).reshape(-1)[:out[n].size])]
    m.close()
    rec = {"steps": nsteps, "io": io, "register": register, "models": models,
           "capture": cap or ("multi" if models >= 4 else "one"),  # virtual: segment graphs per "GPU"
           "dropin_ms_per_step": 1e3 * st["seconds"] / max(1, st["steps_timed"]),
           "graph_ms_per_step": graph_ms, "uploads": st["uploads"], "downloads": st["downloads"],
           "bytes_down": st["bytes_down"],
           "dropin_ms_per_step_steady": float(np.median(st["step_ms"][5:-1])),
           "registered": [ln for ln in r.stderr.splitlines() if ln.startswith("MGCM_AMD: state pages")],
           "host_side_step_ms": [round(x, 4) for x in st["step_ms"]]}
    print("refhost throughput: %s" % json.dumps(rec))
    if os.path.isdir(os.path.join(ROOT, "gpurun_out")):
        with open(os.path.join(ROOT, "gpurun_out", "refhost_throughput_%s_r%d_m%d%s.json" % (io, register, models, "_" + cap if cap else "")), "w") as f:
            json.dump(rec, f)
    assert not bad, bad
    # the state came down after steps 10, 20, ..., 60 (dumpFreq) or after the last only
    assert st["downloads"] == (nsteps // 10 if io == "namelist" else 1) * len(state), st


# BASELINE config 3 through the drop-ins: verification/global_ocean.cs32x15 on the reference's
# own code/SIZE.h (12 tiles of 32 x 16, OL = 4) under pkg/exch2, and on six 32 x 32 tiles (one per
# face, layout "cs32_6t": the device's bench layout).  The harness is built against
# the experiment's headers (build_refhost.py layout "cs32": W2_EXCH2_SIZE.h, staggerTimeStep,
# no CD code) and fills the W2_EXCH2_TOPOLOGY.h COMMON blocks as W2_E2SETUP leaves them
# (W2's default topology: no data.exch2); MGCM_AMD_EXCH2_MAPS hands those arrays to the
# library, which derives the device's halo and vector maps itself (csrc/exch2_maps.hip:
# EXCH2_3D_RL / EXCH2_UV_CGRID_3D_RL restated on point ids).  FORWARD_STEP runs in the
# staggered order (DO_STAGGER_FIELDS_EXCHANGES, then THERMODYNAMICS after the continuity
# step).  The experiment's namelists with nIter0 = 0 (a cold start: the reference tree does
# not hold pickup.0000072000) and taveFreq = 0 (pkg/timeave: refused by the mirror).  Bar: the
# state after 4 steps, with the tiles on 1, 2, 3 and 6 device models (and eager, and the
# device-sharded CG2D), is bit-identical to configs.global_ocean_cs32x15's
# mgcm_forward_step on the same tiling.
CS32_DIR = os.path.join(ROOT, "tests", "golden", "global_ocean.cs32x15", "input")


def _cs32_namelists(dst):
    import re
    os.makedirs(dst, exist_ok=True)
    for fn in ("data", "data.pkg", "data.gmredi"):
        txt = open(os.path.join(CS32_DIR, fn)).read()
        if fn == "data":
            txt, n0 = re.subn(r"(?m)^(\s*)nIter0\s*=\s*\d+\s*,", r"\1nIter0=0,", txt)
            txt, n1 = re.subn(r"(?m)^(\s*)taveFreq\s*=\s*[0-9.eE+]+\s*,", r"\1taveFreq=0.,", txt)
            assert n0 == 1 and n1 == 1, (n0, n1)
        open(os.path.join(dst, fn), "w").write(txt)
    return dst


@pytest.mark.parametrize("layout,models,mwg,eager", [
    ("cs32", 1, 0, 0), ("cs32", 1, 0, 1), ("cs32", 2, 0, 0), ("cs32", 3, 0, 0), ("cs32", 6, 0, 1), ("cs32", 6, 0, 0),
    ("cs32", 3, 1, 0), ("cs32_6t", 1, 0, 0), ("cs32_6t", 2, 0, 0), ("cs32_6t", 3, 0, 0), ("cs32_6t", 6, 0, 0)])
def test_refhost_cs32_exch2_bitexact(layout, models, mwg, eager, tmp_path):
    from mitgcm_amd import configs
    exe = os.path.join(RH, "refhost_" + layout)
    assert os.path.exists(exe), "refhost not built (mitgcm_amd/fortran/build_refhost.py, __graft_entry__.build())"
    nsteps = 4
    sNy = 16 if layout == "cs32" else 32

    def cfg():
        g, params, state, forcing = configs.global_ocean_cs32x15(sNy=sNy)
        if mwg:
            params["cg2dForceMwg"] = 1
        return g, params, state, forcing
    m = configs.make_model(cfg)
    assert (m.g.nSx, m.g.nSy, m.g.sNx, m.g.sNy, m.g.OLx) == (12 if sNy == 16 else 6, 1, 32, sNy, 4)
    pdir = _cs32_namelists(str(tmp_path / "input"))
    w2 = m.g.topo.w2_arrays(ldNb=8, ldT=2 * m.g.nTiles)   # W2_EXCH2_SIZE.h: W2_maxNeighbours, W2_maxNbTiles
    state = _write_blob(tmp_path / "refhost_in.bin", m, nsteps, monitor_days=2, w2=w2, undef=("ALLOW_CD_CODE",))
    env = dict(os.environ, MGCM_AMD_MODELS=str(models), MGCM_CG2D_MWG=str(mwg), MGCM_AMD_EAGER=str(eager))
    r = subprocess.run([exe, str(tmp_path), pdir], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stdout + r.stderr
    out, st = _read_out(tmp_path / "refhost_out.bin", state, nsteps)
    m.forward_step(1)
    m.prepare()
    m.sync()
    t0 = time.perf_counter()
    m.forward_step(nsteps - 1)
    m.sync()
    graph_ms = 1e3 * (time.perf_counter() - t0) / (nsteps - 1)
    bad = [(n, float(np.abs(out[n] - m.get(n).reshape(-1)[:out[n].size]).max())) for n in CHECK
           if n in out and not np.array_equal(out[n], m.get(n).reshape(-1)[:out[n].size])]
    m.close()
    rec = {"layout": layout, "models": models, "cg2dForceMwg": mwg, "eager": eager,
           "dropin_ms_per_step_mean": 1e3 * st["seconds"] / max(1, st["steps_timed"]),
           "dropin_ms_per_step_no_download": st["step_ms"][2], "graph_ms_per_step": graph_ms, "mirror": st,
           "state_fields": len(state)}
    print("refhost %s models=%d mwg=%d eager=%d: %s" % (layout, models, mwg, eager, json.dumps(rec)))
    if os.path.isdir(os.path.join(ROOT, "gpurun_out")):
        with open(os.path.join(ROOT, "gpurun_out", "refhost_%s_m%d_w%d_e%d.json" % (layout, models, mwg, eager)), "w") as f:
            json.dump(rec, f)
    assert not bad, bad
    assert len([n for n in CHECK if n in out]) >= 18
    # the state came down after steps 2 and 4 only (monitorFreq = 2 days, nEndIter = 4)
    assert st["downloads"] == 2 * len(state), (st, len(state))


# BASELINE config 5 (the LLC-90-shaped synthetic, configs.llc_synthetic) through the drop-ins,
# at n = 30: the 5 lat-lon-cap facets as 13 tiles of 30 x 30 (OL = 4, 50 levels) under
# pkg/exch2 (build_refhost.py layout "llc30", refhost/SIZE.h.llc30).  The synthetic has no
# reference experiment, so its namelist is written here from the configuration's own
# parameters (_llc_namelists: each into the group the reference reads it from, refhost_parms.F
# NAMELIST /PARM01/../PARM04/), and refhost resolves it like any other; the W2 arrays are the
# LLC topology's (Exch2Topology.w2_arrays, the facet links with their rotations).  Bars: each
# configured parameter refhost hands the mirror equals the device model's own, and the state
# after 4 steps on 1, 3, 4 and 13 device models (and eager) -- the vector-invariant step with
# C2 tracers, implicit vertical diffusion and IVDC, linear free surface with exactConserv
#  -- is bit-identical to mgcm_forward_step on the same tiling.
LLC_LOGICAL = {"vectorInvariantMomentum", "momDissip_In_AB", "no_slip_sides", "no_slip_bottom", "exactConserv",
               "tempStepping", "tempAdvection", "tempForcing", "saltStepping", "saltAdvection", "saltForcing",
               "implicitDiffusion", "usingCurvilinearGrid"}
LLC_INTEGER = {"selectCoriScheme", "selectVortScheme", "selectKEscheme", "momForcingOutAB", "cg2dMaxIters",
               "cg2dUseMinResSol", "nIter0", "tempAdvScheme", "tempVertAdvScheme", "saltAdvScheme",
               "saltVertAdvScheme", "integr_GeoPot"}


def _namelist_groups():
    """refhost_parms.F's NAMELIST statements: group -> the names it reads."""
    import re
    src = open(os.path.join(RH, "refhost_parms.F")).read()
    groups = {}
    for m in re.finditer(r"NAMELIST /(\w+)/\n((?:     & .*\n)+)", src):
        groups[m.group(1)] = {n.strip() for n in m.group(2).replace("     & ", "").replace("\n", ",").split(",")
                              if n.strip()}
    return groups


def _llc_namelists(dst, params, tRef, sRef, delR, g):
    """data / data.pkg for configs.llc_synthetic's parameters; the CG2D target residual is the
    one its grid's INI_CG2D took (Grid.ini_cg2d: cg2dTargetResidual with the RHS normalised)."""
    os.makedirs(dst, exist_ok=True)
    assert g.cg2dNormaliseRHS and g.cg2dTolerance_sq == 1e-9 * 1e-9
    cg2dTargetResidual = 1e-9
    groups = _namelist_groups()
    fmt = lambda n, v: (".TRUE." if v else ".FALSE.") if n in LLC_LOGICAL else \
        str(int(v)) if n in LLC_INTEGER else repr(float(v))
    body = {g: [] for g in ("PARM01", "PARM02", "PARM03", "PARM04")}
    for n, v in params.items():
        if n == "eosType":
            assert v == 0
            body["PARM01"].append(" eosType='LINEAR',")
            continue
        grp = [g for g in body if n in groups[g]]
        assert len(grp) == 1, (n, grp)
        body[grp[0]].append(" %s=%s," % (n, fmt(n, v)))
    body["PARM01"].append(" tRef=%s," % ", ".join(repr(float(x)) for x in tRef))
    body["PARM01"].append(" sRef=%s," % ", ".join(repr(float(x)) for x in sRef))
    body["PARM01"].append(" implicitFreeSurface=.TRUE.,")
    body["PARM01"].append(" plotLevel=0,")
    body["PARM02"].append(" cg2dTargetResidual=%r," % cg2dTargetResidual)
    body["PARM04"].append(" delR=%s," % ", ".join(repr(float(x)) for x in delR))
    with open(os.path.join(dst, "data"), "w") as f:
        for g, lines in body.items():
            f.write(" &%s\n%s\n &\n\n" % (g, "\n".join(lines)))
    with open(os.path.join(dst, "data.pkg"), "w") as f:
        f.write(" &PACKAGES\n useGMRedi=.FALSE.,\n &\n")
    return dst


@pytest.mark.parametrize("models,eager", [(1, 0), (1, 1), (3, 0), (4, 0), (13, 0)])
def test_refhost_llc30_exch2_bitexact(models, eager, tmp_path):
    from mitgcm_amd import configs
    exe = os.path.join(RH, "refhost_llc30")
    assert os.path.exists(exe), "refhost not built (mitgcm_amd/fortran/build_refhost.py, __graft_entry__.build())"
    nsteps = 4
    out3 = configs.llc_synthetic(n=30)
    g0, params, st0 = out3
    assert (g0.nTiles, g0.sNx, g0.sNy, g0.OLx, g0.Nr) == (13, 30, 30, 4, 50)
    pdir = _llc_namelists(str(tmp_path / "input"), params, st0["tRef"], st0["sRef"], configs.llc_delr(50), g0)
    r = subprocess.run([exe, "--params", pdir, str(tmp_path / "params.txt")], capture_output=True, text=True,
                       timeout=60)
    assert r.returncode == 0, r.stdout + r.stderr
    got = {ln.split()[0]: float(ln.split()[1]) for ln in open(tmp_path / "params.txt")}
    m = configs.make_model(lambda: out3)
    from mitgcm_amd._lib import lib
    skip = ("monitorFreq", "nEndIter", "cg2dNorm", "cg2dTolerance_sq", "cg2dNormaliseRHS")
    # the configuration's own parameters as the device model holds them (the mirror passes
    # every other one too, as the reference resolved it: those the device model left at its
    # defaults are recorded, and the state comparison below is their bar)
    dev = {n: lib().mgcm_get_param(m.h, n.encode()) for n in got if n not in skip}
    pdiff = [(n, got[n], dev[n]) for n in dev if n in params and got[n] != dev[n]]
    pother = [(n, got[n], dev[n]) for n in dev if n not in params and got[n] != dev[n] and dev[n] == dev[n]]
    w2 = m.g.topo.w2_arrays(ldNb=8, ldT=2 * m.g.nTiles)
    state = _write_blob(tmp_path / "refhost_in.bin", m, nsteps, monitor_days=2, w2=w2, undef=("ALLOW_CD_CODE",))
    env = dict(os.environ, MGCM_AMD_MODELS=str(models), MGCM_AMD_EAGER=str(eager))
    r = subprocess.run([exe, str(tmp_path), pdir], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stdout + r.stderr
    out, st = _read_out(tmp_path / "refhost_out.bin", state, nsteps)
    m.forward_step(1)
    m.prepare()
    m.sync()
    t0 = time.perf_counter()
    m.forward_step(nsteps - 1)
    m.sync()
    graph_ms = 1e3 * (time.perf_counter() - t0) / (nsteps - 1)
    bad = [(n, float(np.abs(out[n] - m.get(n).reshape(-1)[:out[n].size]).max())) for n in CHECK
           if n in out and not np.array_equal(out[n], m.get(n).reshape(-1)[:out[n].size])]
    m.close()
    rec = {"layout": "llc30", "models": models, "eager": eager, "params_compared": len(got) - len(skip), "param_diff": pdiff,
           "params_left_at_device_default_resolved_otherwise": pother,
           "dropin_ms_per_step_mean": 1e3 * st["seconds"] / max(1, st["steps_timed"]),
           "graph_ms_per_step": graph_ms, "mirror": st, "state_fields": len(state)}
    print("refhost llc30 models=%d eager=%d: %s" % (models, eager, json.dumps(rec)))
    if os.path.isdir(os.path.join(ROOT, "gpurun_out")):
        with open(os.path.join(ROOT, "gpurun_out", "refhost_llc30_m%d_e%d.json" % (models, eager)), "w") as f:
            json.dump(rec, f)
    assert not pdiff, pdiff
    assert not bad, bad
    assert len([n for n in CHECK if n in out]) >= 18
    assert st["downloads"] == 2 * len(state), (st, len(state))


# The multi-model step captured across the models' own streams (MGCM_AMD_CAPTURE=multi, the
# default from 4 models on: one graph branch per model, joined at every exchange point through
# model 0 -- barrier_all's gather form) against on one stream (MGCM_AMD_CAPTURE=one), with
# every record of the captured step on an event of its own (fortran_abi.hip rec_event):
# bit-identical at 2, 3, 4 and 6 models.  (An all-to-all event barrier captured over 4 or more
# streams makes hipStreamEndCapture fault inside the HIP runtime -- tools/capture_repro.hip
# reproduces it without the library; DESIGN.md section 5, profiles/r06/cap_repro/.)
@pytest.mark.parametrize("layout,models", [("ref", 2), ("ref", 3), ("ref", 4), ("cs32_6t", 3), ("cs32_6t", 6)])
def test_refhost_multistream_capture(layout, models, tmp_path):
    from mitgcm_amd import configs
    exe = os.path.join(RH, "refhost_" + layout)
    assert os.path.exists(exe), "refhost not built (mitgcm_amd/fortran/build_refhost.py, __graft_entry__.build())"
    nsteps = 4
    if layout == "ref":
        m = configs.make_model(lambda: configs.global_ocean_90x40x15(nSx=9, nSy=4))
        state = _write_blob(tmp_path / "refhost_in.bin", m, nsteps, monitor_days=2, packages_off=True)
        pdir = PARAM_DIR
    else:
        m = configs.make_model(lambda: configs.global_ocean_cs32x15(sNy=16 if layout == "cs32" else 32))
        pdir = _cs32_namelists(str(tmp_path / "input"))
        w2 = m.g.topo.w2_arrays(ldNb=8, ldT=2 * m.g.nTiles)
        state = _write_blob(tmp_path / "refhost_in.bin", m, nsteps, monitor_days=2, w2=w2, undef=("ALLOW_CD_CODE",))
    m.close()
    outs, times = {}, {}
    for mode in ("one", "multi"):
        env = dict(os.environ, MGCM_AMD_MODELS=str(models), MGCM_AMD_EAGER="0", MGCM_CG2D_MWG="0",
                   MGCM_AMD_CAPTURE=mode)
        r = subprocess.run([exe, str(tmp_path), pdir], capture_output=True, text=True, timeout=300, env=env)
        assert r.returncode == 0, (mode, r.returncode, r.stdout + r.stderr)
        outs[mode], st = _read_out(tmp_path / "refhost_out.bin", state, nsteps)
        times[mode] = st["step_ms"]
    bad = [n for n in CHECK if n in outs["one"] and not np.array_equal(outs["one"][n], outs["multi"][n])]
    print("refhost %s models=%d step ms one-stream %s multi-stream %s" % (layout, models, times["one"], times["multi"]))
    assert not bad, bad
    assert len(outs["one"]) >= 18


# The drop-ins' multi-GPU path on the one GPU of the test box (MGCM_AMD_DEVICES=virtual: the
# models stand for that many GPUs but all run on device 0): per-GPU CG2D leads, the
# cross-GPU copies of the gathered right-hand side and solution, the halo-source links, and
# the step the drop-ins run when the models span GPUs -- the per-GPU segment graphs replayed
# with event barriers between segments (seg_replay), and routine by routine (MGCM_AMD_EAGER=1)
# -- the code an 8-GPU node runs, bit-identical to one model; mwg = 1: the multi-workgroup
# CG2D launched once per "GPU" on one shared hand-off block.  Both forms' ms/step recorded.
# (the cube's CG2D is the multi-workgroup solve whatever mwg says, and mwg = 1 makes config 2's
# one too: its per-"GPU" launches spin-wait for each other, so they must run together on the one
# device -- with more than two virtual GPUs two of their streams can share one of the process's
# GPU_MAX_HW_QUEUES = 4 hardware queues and serialise; on a real node each GPU has its own)
@pytest.mark.parametrize("layout,models,mwg", [("ref", 2, 0), ("ref", 4, 0), ("ref", 2, 1), ("cs32_6t", 2, 0)])
def test_refhost_virtual_gpus(layout, models, mwg, tmp_path):
    from mitgcm_amd import configs
    exe = os.path.join(RH, "refhost_" + layout)
    assert os.path.exists(exe), "refhost not built (mitgcm_amd/fortran/build_refhost.py, __graft_entry__.build())"
    nsteps = 4

    def cfg():
        if layout == "ref":
            g, params, state, forcing = configs.global_ocean_90x40x15(nSx=9, nSy=4)
        else:
            g, params, state, forcing = configs.global_ocean_cs32x15(sNy=32)
        if mwg:
            params["cg2dForceMwg"] = 1
        return g, params, state, forcing
    m = configs.make_model(cfg)
    if layout == "ref":
        state = _write_blob(tmp_path / "refhost_in.bin", m, nsteps, monitor_days=2, packages_off=True)
        pdir = PARAM_DIR
    else:
        pdir = _cs32_namelists(str(tmp_path / "input"))
        w2 = m.g.topo.w2_arrays(ldNb=8, ldT=2 * m.g.nTiles)
        state = _write_blob(tmp_path / "refhost_in.bin", m, nsteps, monitor_days=2, w2=w2, undef=("ALLOW_CD_CODE",))
    m.close()
    outs, times, nseg = {}, {}, []
    for tag, n, virt, eager in (("one", 1, "0", "0"), ("seg", models, "1", "0"), ("eager", models, "1", "1")):
        env = dict(os.environ, MGCM_AMD_MODELS=str(n), MGCM_CG2D_MWG=str(mwg), MGCM_AMD_EAGER=eager,
                   MGCM_AMD_CAPTURE="debug")
        if virt == "1":
            env["MGCM_AMD_DEVICES"] = "virtual"
        r = subprocess.run([exe, str(tmp_path), pdir], capture_output=True, text=True, timeout=300, env=env)
        assert r.returncode == 0, (tag, r.returncode, r.stdout + r.stderr)
        if tag == "seg":   # the segment graphs were captured and replayed (no fallback to eager)
            assert "segments x %d GPUs" % models in r.stderr and "routine by routine" not in r.stderr, r.stderr[-2000:]
            nseg = [int(ln.split()[2]) for ln in r.stderr.splitlines() if ln.endswith("segments x %d GPUs" % models)]
        outs[tag], st = _read_out(tmp_path / "refhost_out.bin", state, nsteps)
        times[tag] = st["step_ms"]
    bad = [(t, k) for t in ("seg", "eager") for k in CHECK
           if k in outs["one"] and not np.array_equal(outs["one"][k], outs[t][k])]
    rec = {"layout": layout, "virtual_gpus": models, "mwg": mwg, "segments_per_parity": nseg,
           "step_ms_1_model": times["one"],
           "step_ms_segment_graphs": times["seg"], "step_ms_eager": times["eager"]}
    print("refhost virtual GPUs: %s" % json.dumps(rec))
    if os.path.isdir(os.path.join(ROOT, "gpurun_out")):
        with open(os.path.join(ROOT, "gpurun_out", "refhost_vgpu_%s_m%d_w%d.json" % (layout, models, mwg)), "w") as f:
            json.dump(rec, f)
    assert not bad, bad
    assert len(outs["one"]) >= 18
