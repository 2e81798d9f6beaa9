"""The drop-in boundary run the way a reference build runs it: mitgcm_amd/fortran/refhost
(mitgcm_amd/fortran/build_refhost.py) is compiled against the reference's own headers, so
the model state lives in the reference's COMMON blocks (DYNVARS.h, GRID.h, SURFACE.h,
FFIELDS.h, CG2D.h, GMREDI.h, ...), and steps FORWARD_STEP's routine sequence by calling
the MODS shims under their reference names -- DO_OCEANIC_PHYS(myTime, myIter, myThid),
THERMODYNAMICS, DYNAMICS, UPDATE_R_STAR(.TRUE., ...), UPDATE_CG2D, SOLVE_FOR_PRESSURE,
MOMENTUM_CORRECTION_STEP, INTEGR_CONTINUITY(uVel, vVel, ...), CALC_R_STAR(etaH, ...),
DO_FIELDS_BLOCKING_EXCHANGES(myThid) -- with its own EXTERNAL_FIELDS_LOAD in between.  So
MGCM_AMD_MIRROR binds the COMMON blocks and runs, with eosType = 'JMD95P' (BASELINE
config 2's EOS), and the mirror is device-authoritative inside the time loop.

Bars, BASELINE config 2 (global_ocean.90x40x15 from its pickups):
  * on the reference's SIZE.h (9 x 4 tiles of 10 x 10), with the performance CG2D and with
    cg2dRefOrder (the order results/output.txt was summed in, tests/test_gpu_refpin.py),
    and on one 90 x 40 tile: the state after 6 steps through the MODS drop-ins is
    bit-identical to the device-resident, graph-replayed mgcm_forward_step;
  * the same with the 36 tiles over 2, 3 and 4 device models of the one host process
    (MGCM_AMD_MODELS: tiles over GPUs, the models' halo sources and right-hand-side / free-
    surface blocks copied between them at the reference's exchange points), with the gathered
    single-CU CG2D and with the device-sharded multi-workgroup CG2D: bit-identical to one model;
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


def _mirror_calls():
    sys.path.insert(0, os.path.join(ROOT, "mitgcm_amd", "fortran"))
    import build_refhost
    return build_refhost.mirror_calls()


def _name(s):
    return s.encode().ljust(32)


def _write_blob(path, m, nsteps, monitor_days):
    from mitgcm_amd._lib import lib
    L, g = lib(), m.g
    pnames, fields = _mirror_calls()
    dev = {}
    i = 0
    while L.mgcm_param_name(i):
        n = L.mgcm_param_name(i).decode()
        dev[n] = L.mgcm_get_param(m.h, n.encode())
        i += 1
    for n, v in m.params.items():   # options the device reads at set-up beyond its table
        dev.setdefault(n, float(v))
    dtc = dev["deltaTClock"]
    host = {"monitorFreq": monitor_days * dtc, "dumpFreq": 0.0, "chkPtFreq": 0.0, "pChkPtFreq": 0.0,
            "nEndIter": float(int(dev["nIter0"]) + nsteps)}
    params, missing = [], []
    for kind, n in pnames:
        if n in host:
            params.append((n, host[n]))
        elif n in dev:
            params.append((n, float(dev[n])))
        else:
            missing.append(n)
    # parameters this configuration leaves at the reference's default (not in the device's
    # table because no kernel branches on them here)
    assert set(missing) <= {"GM_ExtraDiag", "useAbsVorticity", "upwindShear", "GM_AdvForm", "useSBO",
                            "useDiagnostics"}, missing
    periodic = int(dev.get("periodicExternalForcing", 0))
    nRec = int(dev["nForcRec"]) if periodic else 0
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
                           int(dev["nIter0"]), nRec, periodic], dtype=np.int32).tobytes())
        fh.write(np.array([dtc, dev.get("externForcingPeriod", 0.0), dev.get("externForcingCycle", 0.0)]).tobytes())
        for n, v in params:
            fh.write(_name(n) + np.float64(v).tobytes())
        for n, kind, a in blob_fields:
            fh.write(_name(n) + np.array([a.size, kind], dtype=np.int32).tobytes() + a.tobytes())
        if periodic:
            fh.write(np.ascontiguousarray(m.get("forcRec").reshape(-1)[:6 * nRec * g.nTiles * g.nx * g.ny]).tobytes())
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
@pytest.mark.parametrize("layout,refOrder,models,mwg", [("ref", 0, 1, 0), ("ref", 1, 1, 0), ("1t", 0, 1, 0),
                                                        ("ref", 0, 2, 0), ("ref", 0, 4, 0), ("ref", 1, 4, 0),
                                                        ("ref", 0, 1, 1), ("ref", 0, 3, 1)])
def test_refhost_mods_dropins_bitexact(layout, refOrder, models, mwg, tmp_path):
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
    state = _write_blob(tmp_path / "refhost_in.bin", m, NSTEPS, monitor_days=2)
    env = dict(os.environ, MGCM_CG2D_REFORDER=str(refOrder), MGCM_AMD_MODELS=str(models), MGCM_CG2D_MWG=str(mwg))
    r = subprocess.run([exe, str(tmp_path)], capture_output=True, text=True, timeout=300, env=env)
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
    rec = {"layout": layout, "cg2dRefOrder": refOrder, "models": models, "cg2dForceMwg": mwg,
           "dropin_ms_per_step_mean": ms,
           "dropin_ms_per_step_no_download": float(np.mean(quiet)), "graph_ms_per_step": graph_ms,
           "mirror": st, "state_fields": len(state)}
    print("refhost %s refOrder=%d models=%d mwg=%d: %s" % (layout, refOrder, models, mwg, json.dumps(rec)))
    if os.path.isdir(os.path.join(ROOT, "gpurun_out")):
        with open(os.path.join(ROOT, "gpurun_out", "refhost_%s_%d_m%d_w%d.json" % (layout, refOrder, models, mwg)),
                  "w") as f:
            json.dump(rec, f)
    assert not bad, bad
    assert len([n for n in CHECK if n in out]) >= 20
    # the state came down after steps 2, 4 and 6 only (monitorFreq = 2 days, nEndIter = 6)
    assert st["downloads"] == 3 * len(state), (st, len(state))
