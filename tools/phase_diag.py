"""Phase-1 outputs of a single-tile range against the whole-domain phase 1 (one process).
python tools/phase_diag.py [ntile-per-range]"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mitgcm_amd import configs  # noqa: E402
from mitgcm_amd._lib import lib  # noqa: E402

F = ("Kwx", "Kwy", "Kwz", "Kux", "Kvy", "Kuz", "Kvz", "GM_PsiX", "GM_PsiY", "rhoInSitu", "sigmaR", "gU", "gV", "guNm1",
     "gvNm1", "cg2d_b", "surfaceForcingT", "PmEpR", "IVDConvCount")
L = lib()
nt = int(sys.argv[1]) if len(sys.argv) > 1 else 1


def run(t0, n):
    m = configs.make_model(configs.global_ocean_cs32x15)
    if n:
        L.mgcm_set_tile_range(m.h, t0, n)
    L.mgcm_begin_steps(m.h)
    assert L.mgcm_step_phase(m.h, 1) == 0
    m.sync()
    out = {}
    for f in F:
        try:
            out[f] = m.get(f)
        except Exception:
            pass
    m.close()
    return out


full = run(0, 0)
for t0 in range(0, 6 - nt + 1):
    o = run(t0, nt)
    for f, a in o.items():
        b = full[f]
        for t in range(t0, t0 + nt):
            if not np.array_equal(a[t], b[t], equal_nan=True):
                d = np.abs(a[t] - b[t])
                w = np.argwhere(d > 0)
                print("range(%d,%d) %-10s tile %d: %d points, max %.3g, first %s" % (t0, nt, f, t, len(w), np.nanmax(d),
                                                                              w[:3].tolist()), flush=True)
print("done")
