"""WRITE_PICKUP (model/src/write_pickup.F:107-322) and CD_CODE_WRITE_PICKUP
(pkg/cd_code/cd_code_write_pickup.F) for the device model: the state the next run needs
to restart bit for bit, downloaded once at checkpoint time and written as the
reference's MDS pickup -- global big-endian fp64 records (MDS_WRITE_FIELD with
globalFiles) plus the `.meta` text of MDS_WR_METAFILES (pkg/mdsio/mds_wr_metafiles.F).

Record order (write_pickup.F, ALLOW_ADAMSBASHFORTH_3 undefined):
  Uvel, Vvel, Theta, Salt                           Nr records each
  GuNm1, GvNm1 (momStepping)                        Nr each
  GtNm1 / GsNm1 (AB2 on the tracer tendency: C2)     Nr each
  PhiHyd (storePhiHyd4Phys: totPhiHyd)              Nr
  EtaN, dEtaHdt, EtaH (= etaHnm1, update_etah.F:52)  1 record each (EXACT_CONSERV)
pickup_cd (useCDscheme): uVelD, vVelD, uNM1, vNM1 (Nr each), etaNm1 (1).

read_pickup() (configs.py) reads both back; the round trip of the reference's own
pickup.0000036000 reproduces its bytes (tests/test_pickup.py), and a device run
restarted from a written pickup continues bit for bit (tests/test_gpu_restart.py,
the verification/testreport tst_2+2 check)."""
import os

import numpy as np


def tiles_to_global(g, arr):
    """Tile layout (..., nTiles, ny, nx) -> the global MDS array (..., Ny, Nx), interiors.
    Lat-lon tilings: tiles (bi, bj) in an nSx x nSy grid (the inverse of configs._to_tiles).
    EXCH2 (cube / LLC) tilings: W2_mapIO = -1, the facets one after the other in x
    (w2_set_map_tiles.F:136-205, the inverse of configs.cs_global_to_tiles(mapIO=-1))."""
    arr = np.asarray(arr)
    lead = arr.shape[:-3]
    inner = g.sl(1, g.sNx, 1, g.sNy)
    topo = getattr(g, "topo", None)
    if topo is not None and hasattr(topo, "facet_dims"):
        Nx = sum(fx for fx, _ in topo.facet_dims)
        Ny = max(fy for _, fy in topo.facet_dims)
        out = np.zeros(lead + (Ny, Nx))
        for t in range(g.nTiles):
            tid = t + 1
            f = topo.face[tid]
            x0 = sum(fx for fx, _ in topo.facet_dims[:f - 1]) + topo.tBx[tid]
            y0 = topo.tBy[tid]
            out[..., y0:y0 + g.sNy, x0:x0 + g.sNx] = arr[(Ellipsis, t) + inner]
        return out
    out = np.zeros(lead + (g.sNy * g.nSy, g.sNx * g.nSx))
    for t in range(g.nTiles):
        bi, bj = t % g.nSx, t // g.nSx
        out[..., bj * g.sNy:(bj + 1) * g.sNy, bi * g.sNx:(bi + 1) * g.sNx] = arr[(Ellipsis, t) + inner]
    return out


def pickup_records(params):
    """The (name, 3-D?, MDS field name) list WRITE_PICKUP writes for these run parameters."""
    p = params
    recs = [("uVel", True, "Uvel"), ("vVel", True, "Vvel"), ("theta", True, "Theta"), ("salt", True, "Salt")]
    if p.get("momStepping", 1):
        recs += [("guNm1", True, "GuNm1"), ("gvNm1", True, "GvNm1")]
    # AdamsBashforthGt/Gs: AB2 on the tendency, i.e. the C2 scheme (gad_init_fixed.F:126-162)
    if p.get("tempStepping", 1) and p.get("tempAdvScheme", 2) == 2:
        recs.append(("gtNm1", True, "GtNm1"))
    if p.get("saltStepping", 1) and p.get("saltAdvScheme", 2) == 2:
        recs.append(("gsNm1", True, "GsNm1"))
    if p.get("storePhiHyd4Phys", 0):
        recs.append(("totPhiHyd", True, "PhiHyd"))
    recs.append(("etaN", False, "EtaN"))
    recs += [("dEtaHdt", False, "dEtaHdt"), ("etaHnm1", False, "EtaH")]
    return recs


def write_meta(path, simulation, Nx, Ny, nrec, myIter, myTime, flds):
    """MDS_WR_METAFILES (pkg/mdsio/mds_wr_metafiles.F) for a global 2-D-record file."""
    lines = [" simulation = { '%s' };" % simulation,
             " nDims = [%4d ];" % 2,
             " dimList = [",
             "%6d,%5d,%5d," % (Nx, 1, Nx),
             "%6d,%5d,%5d" % (Ny, 1, Ny),
             " ];",
             " dataprec = [ 'float64' ];",
             " nrecords = [%6d ];" % nrec,
             " timeStepNumber = [%11d ];" % myIter,
             " timeInterval = [%20.12E ];" % myTime]
    if flds:
        lines += [" nFlds = [%5d ];" % len(flds), " fldList = {",
                  " " + " ".join("'%-8s'" % f for f in flds), " };"]
    with open(path, "w") as fh:
        fh.write("\n".join(lines) + "\n")


def write_pickup_fields(g, params, fields, directory, myIter, myTime, simulation="mitgcm_amd", cd=None):
    """Write pickup.<iter>.data/.meta (and pickup_cd.<iter>.data/.meta when cd is given) from
    tile-layout host arrays: fields[name] (nTiles, Nr, ny, nx) for 3-D, (nTiles, ny, nx) for 2-D."""
    recs = pickup_records(params)
    blocks = []
    for name, is3d, _ in recs:
        a = np.asarray(fields[name], dtype=np.float64)
        glob = tiles_to_global(g, np.moveaxis(a, 0, 1) if is3d else a)   # (Nr, Ny, Nx) / (Ny, Nx)
        blocks.append(glob.reshape((-1,) + glob.shape[-2:]))
    data = np.concatenate(blocks)
    Ny, Nx = data.shape[-2:]
    base = os.path.join(directory, "pickup.%010d" % myIter)
    data.astype(">f8").tofile(base + ".data")
    write_meta(base + ".meta", simulation, Nx, Ny, data.shape[0], myIter, myTime, [r[2] for r in recs])
    if cd is not None:
        blocks = [tiles_to_global(g, np.moveaxis(np.asarray(cd[n], dtype=np.float64), 0, 1))
                  for n in ("uVelD", "vVelD", "uNM1", "vNM1")]
        blocks.append(tiles_to_global(g, np.asarray(cd["etaNm1"], dtype=np.float64))[None])
        data = np.concatenate(blocks)
        base = os.path.join(directory, "pickup_cd.%010d" % myIter)
        data.astype(">f8").tofile(base + ".data")
        write_meta(base + ".meta", simulation, Nx, Ny, data.shape[0], myIter, myTime, None)
    return base


def write_pickup(model, directory, simulation="mitgcm_amd"):
    """WRITE_PICKUP of a device model at its current step: one download of the restart
    state (model.get), then the MDS files.  Returns myIter."""
    model.sync()
    myIter = model.my_iter()
    myTime = myIter * model.params["deltaTClock"]
    p = model.params
    names = [r[0] for r in pickup_records(p)]
    fields = {n: model.get(n) for n in names}
    cd = None
    if p.get("useCDscheme", 0):
        cd = {n: model.get(n) for n in ("uVelD", "vVelD", "uNM1", "vNM1", "etaNm1")}
    write_pickup_fields(model.g, p, fields, directory, myIter, myTime, simulation, cd)
    return myIter
