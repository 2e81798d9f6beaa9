"""Host-side spherical-polar grid (INI_SPHERICAL_POLAR_GRID, INI_CORI map 2)
against the grid statistics the reference prints at start-up
(model/src/ini_grid.F:128-145, MON_STATS_RS pkg/monitor/mon_stats_rs.F), from
the committed verification/tutorial_baroclinic_gyre/results/output.txt."""
import json
import os

import numpy as np

from conftest import digits


def mon_stats_rs(g, a):
    """MON_STATS_RS: unweighted min/max/mean/sd over tile interiors, tile-ordered sums."""
    inner = g.sl(1, g.sNx, 1, g.sNy)
    vals = [a[t][inner] for t in range(g.nTiles)]
    tm, tv, n = [], [], 0
    for v in vals:
        s = s2 = 0.0
        for x in v.ravel():
            s = s + x
            s2 = s2 + x * x
        tm.append(s); tv.append(s2); n += v.size
    mean = sum(tm, 0.0) * (1.0 / n)
    sd = 0.0
    for v in vals:
        st = 0.0
        for x in v.ravel():
            st = st + (x - mean) * (x - mean)
        sd = sd + st
    sd = np.sqrt(sd * (1.0 / n))
    allv = np.concatenate([v.ravel() for v in vals])
    return {"max": allv.max(), "min": allv.min(), "mean": mean, "sd": sd}


def test_baroclinic_grid_matches_reference_printout(golden_dir):
    from mitgcm_amd import configs
    g, params, state = configs.baroclinic_gyre()
    gold = json.load(open(os.path.join(golden_dir, "tutorial_baroclinic_gyre", "grid_monitor.json")))
    names = {"XC": "xC", "XG": "xG", "DXC": "dxC", "DXF": "dxF", "DXG": "dxG", "DXV": "dxV", "YC": "yC",
             "YG": "yG", "DYC": "dyC", "DYF": "dyF", "DYG": "dyG", "DYU": "dyU", "RA": "rA", "RAW": "rAw",
             "RAS": "rAs", "RAZ": "rAz", "fCori": "fCori", "fCoriG": "fCoriG", "fCoriCos": "fCoriCos"}
    worst = (99.0, None)
    for mon, f in names.items():
        st = mon_stats_rs(g, g.f[f])
        for k in ("max", "min", "mean", "sd"):
            ref = gold["%s_%s" % (mon, k)]
            if k == "sd" and abs(ref) < 1e-6 * max(abs(gold["%s_max" % mon]), 1e-30):
                continue       # sd of a constant field: roundoff-level, not meaningful
            d = digits(st[k], ref)
            if d < worst[0]:
                worst = (d, (mon, k, st[k], ref))
    assert worst[0] >= 12.5, worst
