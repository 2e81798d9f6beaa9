"""BASELINE config 2 on the device, pinned to the reference's own committed output.

verification/global_ocean.90x40x15/results/output.txt was produced on the reference's
tiling (code/SIZE.h: 9 x 4 tiles of 10 x 10, OL = 3).  The device runs that tiling here
with cg2dRefOrder = 1: CG2D's dot products are summed in the reference's order -- per tile
sequentially (j outer, i inner, cg2d.F:211-243,268-296,305-337), the tile partials in
global tile order (GLOBAL_SUM_TILE_RL, global_sum_tile.F:161-191) -- and the operator rows
in cg2d.F's operand order without fused multiply-adds.

Bars (SURVEY.md 8(c) items 3-4, 10 steps from pickup.0000036000):
  * against the oracle in the reference's summation order on the same 36 tiles: every
    CG2D residual and iteration count and the state arrays bit-identical;
  * against results/output.txt: >= 13 digits (testreport's formula) on every dynstat
    value and CG2D residual the monitor prints, cg2d_iters identical every step.
The performance path (one 90 x 40 tile, the FMA/tree-order CG2D of bench.py) is pinned
by test_gpu_ocean90.py; its digits against output.txt are recorded there.
"""
import json
import os

import numpy as np
import pytest

from conftest import digits

pytestmark = pytest.mark.gpu
EXP = "global_ocean.90x40x15"
STATE = ("uVel", "vVel", "wVel", "theta", "salt", "etaN", "etaH", "guNm1", "gvNm1", "gtNm1", "gsNm1", "totPhiHyd")


def _cfg():
    from mitgcm_amd import configs
    g, params, state, forcing = configs.global_ocean_90x40x15(nSx=9, nSy=4)
    params["cg2dRefOrder"] = 1
    return g, params, state, forcing


def test_ocean90_reference_tiling_pinned_to_output_txt(golden_dir):
    from mitgcm_amd import configs
    from mitgcm_amd.model import dynstat
    from oracle.harness import ocean90_oracle
    m = configs.make_model(_cfg)
    assert m.cg2d_kernel() == "block_ref"
    assert m.g.nTiles == 36 and (m.g.sNx, m.g.sNy) == (10, 10)
    o, g = ocean90_oracle(nSx=9, nSy=4)
    gold = json.load(open(os.path.join(golden_dir, EXP, "monitor.json")))
    worst = (99.0, None)
    for step in range(1, 11):
        m.forward_step(1)
        o.forward_step()
        md = m.solve_stats()
        od = o.dynstat()
        # the solve: bit-identical to the reference-order oracle
        for k in ("cg2d_init_res", "cg2d_last_res", "cg2d_iters"):
            assert md[k] == od[k], ("oracle", step, k, md[k], od[k])
        md.update(dynstat(m))
        ref = gold[step]
        assert md["cg2d_iters"] == ref["cg2d_iters"], (step, md["cg2d_iters"], ref["cg2d_iters"])
        for k, v in md.items():
            if k in ref and k != "cg2d_iters":
                worst = min(worst, (digits(v, ref[k]), (step, k, v, ref[k])))
    inner = (Ellipsis,) + g.sl(1, g.sNx, 1, g.sNy)
    bad = []
    for n in STATE:
        dev = m.get(n)
        orc = np.array(o.arr(n)).reshape(dev.shape)
        if not np.array_equal(dev[inner], orc[inner]):
            bad.append((n, float(np.abs(dev - orc)[inner].max())))
    m.close()
    print("global_ocean.90x40x15 on 36 tiles, cg2dRefOrder: vs results/output.txt worst %.2f digits at %s"
          % worst)
    assert not bad, bad
    assert worst[0] >= 13.0, worst
