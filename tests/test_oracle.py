"""The oracle (CPU restatement, oracle/*.c) pinned against the reference's own
committed output: verification/tutorial_barotropic_gyre/results/output.txt,
parsed into tests/golden/tutorial_barotropic_gyre/monitor.json."""
import json
import os

import numpy as np
import pytest

from conftest import digits
from oracle.harness import gyre_oracle


def test_gyre_params_pinned(golden_dir):
    """Parameters the oracle assumes == the reference's resolved configuration dump."""
    p = json.load(open(os.path.join(golden_dir, "tutorial_barotropic_gyre", "params.json")))
    assert float(p["deltaTMom"]) == 1200.0 and float(p["deltaTFreeSurf"]) == 1200.0
    assert float(p["abEps"]) == 0.01 and int(p["momForcingOutAB"]) == 0
    assert p["momDissip_In_AB"] == "T" and p["no_slip_sides"] == "T"
    assert float(p["sideDragFactor"]) == 2.0 and float(p["rhoConst"]) == 1000.0
    assert int(p["cg2dUseMinResSol"]) == 0 and int(p["cg2dMaxIters"]) == 1000
    assert p["useEnergyConservingCoriolis"] == "F" and p["useJamartWetPoints"] == "F"
    assert float(p["globalArea"]) == 1.44e12


def test_gyre_oracle_matches_reference_output(golden_dir):
    gold = json.load(open(os.path.join(golden_dir, "tutorial_barotropic_gyre", "monitor.json")))
    o = gyre_oracle()
    assert o.get("globalArea") == 1.44e12
    assert abs(o.get("cg2dNorm") - 2.0e-4) < 1e-20
    for n in range(1, 11):
        o.forward_step()
        r = o.dynstat()
        g = gold[n]
        assert r["cg2d_iters"] == g["cg2d_iters"], n
        for k, v in r.items():
            if k in g and k != "cg2d_iters":
                # the reference prints 14 significant digits: >= 13 digits is print precision
                assert digits(v, g[k]) >= 13.0, (n, k, v, g[k])
