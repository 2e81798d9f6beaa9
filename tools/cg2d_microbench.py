"""CG2D per-iteration latency on synthetic cartesian grids (closed basin, flat
bottom): runs the device solver for a fixed iteration count (tolerance 0) and
reports microseconds per CG iteration from the kernel's HIP-event duration."""
import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mitgcm_amd.grid import Grid  # noqa: E402
from mitgcm_amd.model import Model  # noqa: E402


def make(sNx, sNy, nSx=1, nSy=1, OL=2, Nr=1):
    g = Grid(sNx, sNy, OL, OL, Nr, nSx, nSy)
    g.ini_vertical_grid([1000.0] * Nr)
    Nx, Ny = sNx * nSx, sNy * nSy
    g.ini_cartesian_grid(np.full(Nx, 1e4), np.full(Ny, 1e4), 0.0, 0.0)
    g.ini_cori(1e-4, 1e-11)
    bathy = np.full((Ny, Nx), -1000.0 * Nr)
    bathy[0, :] = bathy[-1, :] = 0.0
    bathy[:, 0] = bathy[:, -1] = 0.0
    g.ini_depths_masks(bathy)
    g.ini_cg2d(1200.0, 1200.0, 0.0)
    return g


def run(sNx, sNy, nSx=1, nSy=1, iters=400):
    g = make(sNx, sNy, nSx, nSy)
    m = Model(g, dict(cg2dMaxIters=iters))
    m.init()
    rng = np.random.default_rng(0)
    b = rng.standard_normal((g.nTiles, g.ny, g.nx)) * g.f["maskInC"]
    x = np.zeros_like(b)
    m.cg2d(b, x, iters)  # warm
    m.kernel_timing(True)
    reps = 5
    for _ in range(reps):
        out = m.cg2d(b, x, iters)
    ms, n = m.kernel_ms("cg2d")
    m.kernel_timing(False)
    its = out[4]
    m.close()
    return {"grid": [sNx, sNy, nSx * nSy], "points": g.nTiles * sNx * sNy, "iters": its,
            "us_per_iter": 1e3 * ms / its, "launch_ms": ms}


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=400)
    a = ap.parse_args()
    res = []
    for (sx, sy, tx, ty) in [(30, 30, 1, 1), (62, 62, 1, 1), (90, 40, 1, 1), (32, 32, 2, 2), (32, 32, 3, 2), (90, 90, 1, 1)]:
        r = run(sx, sy, tx, ty, a.iters)
        r["creg"] = os.environ.get("MGCM_CG2D_CREG", "default")
        res.append(r)
        print(json.dumps(r), flush=True)
